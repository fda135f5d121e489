// Exact emulation of libstdc++'s std::sort (introsort, _S_threshold = 16, median-of-three,
// unguarded partition, heap-sort fallback at depth 2*lg(n), final insertion sort) for the
// comparator used by QuadTreeSuppression: `lhs.size > rhs.size` (src/ORBextractor.cc:642-643).
//
// std::sort is unstable, so which of several equal-size nodes is split first — and therefore the
// quadtree's output — depends on the library's exact move sequence.  This header reproduces that
// sequence element-for-element; tests/test_qt_sort.py checks it against the real std::sort.
//
// Usable from host code (tests) and device code (the quadtree kernel's serial section).
#pragma once

#if defined(__HIPCC__)
#define QT_HD __host__ __device__ __forceinline__
#else
#define QT_HD inline
#endif

namespace orbamd {

struct QtItem {
    int size;  // DivisibleNode::size
    int node;  // DivisibleNode::ptr (node position)
};

// comp(a, b) == a.size > b.size
QT_HD bool qt_less(const QtItem& a, const QtItem& b) { return a.size > b.size; }

QT_HD void qt_swap(QtItem* a, QtItem* b) {
    QtItem t = *a;
    *a = *b;
    *b = t;
}

QT_HD int qt_lg(int n) {  // std::__lg
    int r = 0;
    while (n > 1) {
        n >>= 1;
        ++r;
    }
    return r;
}

// std::__move_median_to_first(result, a, b, c)
QT_HD void qt_median_to_first(QtItem* result, QtItem* a, QtItem* b, QtItem* c) {
    if (qt_less(*a, *b)) {
        if (qt_less(*b, *c)) qt_swap(result, b);
        else if (qt_less(*a, *c)) qt_swap(result, c);
        else qt_swap(result, a);
    } else if (qt_less(*a, *c)) qt_swap(result, a);
    else if (qt_less(*b, *c)) qt_swap(result, c);
    else qt_swap(result, b);
}

// std::__unguarded_partition(first, last, pivot)
QT_HD QtItem* qt_unguarded_partition(QtItem* first, QtItem* last, QtItem* pivot) {
    while (true) {
        while (qt_less(*first, *pivot)) ++first;
        --last;
        while (qt_less(*pivot, *last)) --last;
        if (!(first < last)) return first;
        qt_swap(first, last);
        ++first;
    }
}

// std::__push_heap(first, holeIndex, topIndex, value)
QT_HD void qt_push_heap(QtItem* first, int hole, int top, QtItem value) {
    int parent = (hole - 1) / 2;
    while (hole > top && qt_less(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

// std::__adjust_heap(first, holeIndex, len, value)
QT_HD void qt_adjust_heap(QtItem* first, int hole, int len, QtItem value) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (qt_less(first[second], first[second - 1])) second--;
        first[hole] = first[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        first[hole] = first[second - 1];
        hole = second - 1;
    }
    qt_push_heap(first, hole, top, value);
}

// std::__make_heap + std::__sort_heap  (== std::__partial_sort(first, last, last))
QT_HD void qt_heap_sort(QtItem* first, QtItem* last) {
    const int len = (int)(last - first);
    if (len >= 2) {
        int parent = (len - 2) / 2;
        while (true) {
            QtItem v = first[parent];
            qt_adjust_heap(first, parent, len, v);
            if (parent == 0) break;
            parent--;
        }
    }
    while (last - first > 1) {
        --last;
        QtItem v = *last;  // std::__pop_heap(first, last, last)
        *last = *first;
        qt_adjust_heap(first, 0, (int)(last - first), v);
    }
}

// std::__unguarded_linear_insert(last)
QT_HD void qt_unguarded_linear_insert(QtItem* last) {
    QtItem val = *last;
    QtItem* next = last - 1;
    while (qt_less(val, *next)) {
        *last = *next;
        last = next;
        --next;
    }
    *last = val;
}

// std::__insertion_sort(first, last)
QT_HD void qt_insertion_sort(QtItem* first, QtItem* last) {
    if (first == last) return;
    for (QtItem* i = first + 1; i != last; ++i) {
        if (qt_less(*i, *first)) {
            QtItem val = *i;
            for (QtItem* p = i; p != first; --p) *p = *(p - 1);  // move_backward
            *first = val;
        } else {
            qt_unguarded_linear_insert(i);
        }
    }
}

// std::__introsort_loop — the recursion on the right part is made iterative with an explicit
// stack; the visiting order (right part first, then loop on the left part) is unchanged.
QT_HD void qt_introsort_loop(QtItem* first0, QtItem* last0, int depth0) {
    struct Frame {
        QtItem* first;
        QtItem* last;
        int depth;
    };
    Frame stack[64];
    int sp = 0;
    stack[sp++] = Frame{first0, last0, depth0};
    while (sp > 0) {
        Frame f = stack[--sp];
        QtItem* first = f.first;
        QtItem* last = f.last;
        int depth = f.depth;
        // Executing the original loop body; a recursive call becomes "push the rest of this
        // frame, then run the callee first".
        while (last - first > 16) {
            if (depth == 0) {
                qt_heap_sort(first, last);
                last = first;  // return
                break;
            }
            --depth;
            QtItem* mid = first + (last - first) / 2;
            qt_median_to_first(first, first + 1, mid, last - 1);
            QtItem* cut = qt_unguarded_partition(first + 1, last, first);
            // std::__introsort_loop(cut, last, depth); then last = cut and continue.
            stack[sp++] = Frame{first, cut, depth};  // continuation of this frame (runs later)
            stack[sp++] = Frame{cut, last, depth};   // recursive call (runs next)
            first = last;                            // end this activation
            break;
        }
    }
}

// std::sort(first, last, comp)
QT_HD void qt_sort(QtItem* first, QtItem* last) {
    const int n = (int)(last - first);
    if (n <= 0) return;
    qt_introsort_loop(first, last, 2 * qt_lg(n));
    if (n > 16) {
        qt_insertion_sort(first, first + 16);
        for (QtItem* i = first + 16; i != last; ++i) qt_unguarded_linear_insert(i);
    } else {
        qt_insertion_sort(first, last);
    }
}

// ------------------------------------------------------------------------------------------
// Data-parallel formulation of the same sort (what the quadtree kernel runs on a wavefront).
//
//  * __unguarded_partition(first+1, last, pivot=first) with p = pivot.size: let Ls = ascending
//    positions in [first+1, last) with size <= p (left-scan stops) and Rs = descending positions
//    in [first, last) with size >= p (right-scan stops), both in the array as it stands before
//    the partition.  The k-th swap exchanges Ls[k] and Rs[k] for every k with Ls[k] < Rs[k]
//    (a prefix of k, K of them), and the returned cut is Ls[0] when K == 0, otherwise
//    min(Ls[K], Rs[K-1]).  (Positions strictly between the k-th stops are untouched by earlier
//    swaps, so each scan's next stop is the next original stopper or the nearest swapped slot.)
//  * __final_insertion_sort is a stable insertion sort, and introsort_loop leaves the array as a
//    sequence of final segments (<= 16 elements, or heap-sorted) with every element of a segment
//    >= every element of any later segment; so the insertion pass is a stable sort inside each
//    final segment.
// qt_sort_parallel_form() is the sequential statement of that formulation, checked against
// std::sort by tests/native/qt_sort_check.cpp.
// ------------------------------------------------------------------------------------------
QT_HD int qt_partition_parallel_form(QtItem* a, int lo, int hi, int* Ls, int* Rs) {
    const int p = a[lo].size;
    int nl = 0, nr = 0;
    for (int i = lo + 1; i < hi; i++)
        if (a[i].size <= p) Ls[nl++] = i;
    for (int j = hi - 1; j >= lo; j--)
        if (a[j].size >= p) Rs[nr++] = j;
    int K = 0;
    while (K < nl && K < nr && Ls[K] < Rs[K]) K++;
    for (int k = 0; k < K; k++) qt_swap(&a[Ls[k]], &a[Rs[k]]);
    if (K == 0) return Ls[0];
    const int c1 = K < nl ? Ls[K] : hi;
    return c1 < Rs[K - 1] ? c1 : Rs[K - 1];
}

// seg_lo[i] / seg_len[i]: final segment of position i (seg_len < 0: heap-sorted segment).
QT_HD void qt_sort_parallel_form(QtItem* a, int n, int* Ls, int* Rs, int* seg_lo, int* seg_len, QtItem* tmp) {
    if (n <= 0) return;
    struct Frame { int lo, hi, depth; };
    Frame stack[64];
    int sp = 0;
    stack[sp++] = Frame{0, n, 2 * qt_lg(n)};
    while (sp > 0) {
        Frame f = stack[--sp];
        int lo = f.lo, hi = f.hi, depth = f.depth;
        if (hi - lo > 16) {
            if (depth == 0) {
                qt_heap_sort(a + lo, a + hi);
                for (int i = lo; i < hi; i++) { seg_lo[i] = lo; seg_len[i] = -1; }
                continue;
            }
            --depth;
            const int mid = lo + (hi - lo) / 2;
            qt_median_to_first(a + lo, a + lo + 1, a + mid, a + hi - 1);
            const int cut = qt_partition_parallel_form(a, lo, hi, Ls, Rs);
            stack[sp++] = Frame{lo, cut, depth};
            stack[sp++] = Frame{cut, hi, depth};
            continue;
        }
        for (int i = lo; i < hi; i++) { seg_lo[i] = lo; seg_len[i] = hi - lo; }
    }
    // stable sort inside each final segment (descending size)
    for (int i = 0; i < n; i++) {
        if (seg_len[i] < 0) { tmp[i] = a[i]; continue; }
        const int lo = seg_lo[i], hi = lo + seg_len[i];
        int r = 0;
        for (int j = lo; j < hi; j++)
            r += (a[j].size > a[i].size) || (a[j].size == a[i].size && j < i);
        tmp[lo + r] = a[i];
    }
    for (int i = 0; i < n; i++) a[i] = tmp[i];
}

}  // namespace orbamd
