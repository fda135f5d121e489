"""ORBVocabulary mirror (DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>, include/ORBVocabulary.h)
over the gfx950 C-ABI: loadFromTextFile and transform(features, BowVector&, FeatureVector&, levelsup)
(Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1130-1263, :1341-1431)."""
import ctypes as C

import numpy as np

from ._lib import check, lib, ptr, stream_ptr, tptr

TF_IDF, TF, IDF, BINARY = 0, 1, 2, 3                                   # BowVector.h WeightingType
L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT = range(6)  # BowVector.h ScoringType


class ORBVocabulary:
    def __init__(self, handle, device):
        self._h = handle
        self.device = device

    @classmethod
    def loadFromTextFile(cls, path, device: int = 0) -> "ORBVocabulary":
        h = C.c_void_p()
        check(lib().orbv_load_text(str(path).encode(), device, C.byref(h)), "orbv_load_text")
        return cls(h, device)

    @classmethod
    def from_arrays(cls, k, L, scoring, weighting, parent, is_leaf, desc, weight, device: int = 0) -> "ORBVocabulary":
        parent = np.ascontiguousarray(parent, np.int32)
        is_leaf = np.ascontiguousarray(is_leaf, np.uint8)
        desc = np.ascontiguousarray(desc, np.uint8)
        weight = np.ascontiguousarray(weight, np.float64)
        h = C.c_void_p()
        check(lib().orbv_create(k, L, scoring, weighting, len(parent), ptr(parent), ptr(is_leaf), ptr(desc), ptr(weight),
                                device, C.byref(h)), "orbv_create")
        return cls(h, device)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orbv_destroy(self._h)
            self._h = None

    def info(self) -> dict:
        v = [C.c_int() for _ in range(6)]
        check(lib().orbv_info(self._h, *[C.byref(x) for x in v]), "orbv_info")
        return dict(zip(("k", "L", "n_nodes", "n_words", "scoring", "weighting"), (x.value for x in v)))

    def transform(self, descriptors, levelsup: int = 4):
        """Returns (BowVector as (word ids, weights) ascending, FeatureVector as (node ids, offsets, indices))."""
        d = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        n = len(d)
        cap = max(n, 1)
        bw, bv = np.zeros(cap, np.uint32), np.zeros(cap)
        fn, fo, fi = np.zeros(cap, np.uint32), np.zeros(cap + 1, np.int32), np.zeros(cap, np.int32)
        nw, nn = C.c_int(), C.c_int()
        check(lib().orbv_transform(self._h, ptr(d), n, levelsup, ptr(bw), ptr(bv), C.byref(nw), ptr(fn), ptr(fo),
                                   ptr(fi), C.byref(nn)), "orbv_transform")
        return (bw[:nw.value], bv[:nw.value]), (fn[:nn.value], fo[:nn.value + 1], fi[:fo[nn.value]])

    def transform_batch_device(self, desc, counts, levelsup: int = 4, out=None, stream=None):
        """desc: (F, cap, 32) uint8 CUDA tensor, counts: (F,) int32 (an extract_batch_device output)."""
        import torch
        F, cap = int(desc.shape[0]), int(desc.shape[1])
        dev = desc.device
        if out is None:
            out = dict(bow_word=torch.empty((F, cap), dtype=torch.int32, device=dev),
                       bow_weight=torch.empty((F, cap), dtype=torch.float64, device=dev),
                       n_words=torch.empty(F, dtype=torch.int32, device=dev),
                       fv_node=torch.empty((F, cap), dtype=torch.int32, device=dev),
                       fv_off=torch.empty((F, cap + 1), dtype=torch.int32, device=dev),
                       fv_idx=torch.empty((F, cap), dtype=torch.int32, device=dev),
                       n_nodes=torch.empty(F, dtype=torch.int32, device=dev))
        check(lib().orbv_transform_batch_device(self._h, tptr(desc), tptr(counts), cap, F, levelsup,
                                                tptr(out["bow_word"]), tptr(out["bow_weight"]), tptr(out["n_words"]),
                                                tptr(out["fv_node"]), tptr(out["fv_off"]), tptr(out["fv_idx"]),
                                                tptr(out["n_nodes"]), stream_ptr(stream)),
              "orbv_transform_batch_device")
        return out
