#!/bin/bash
# One GPU session, parameterised: the steps named on the command line run in order, each GPU step under
# its own time limit; the chain stops at the first failure and nothing runs on the GPU after it.
#
#   tests    the whole -m gpu suite            xtests   extractor / drop-in / matcher tests only
#   pjk1     SearchByProjection tests against the K = 1 diagnostic build (every claim takes the rescan)
#   smoke    __graft_entry__.smoke()           det      tools/diag/desc_determinism.py (describe, 5 runs)
#   bench    bench.py $BENCH_ARGS              ba_ab    tools/babench.py, tools/ab/lib_$BASE.so vs in-tree
#   kb_pan | kb_tex   tools/kbench.py, tools/ab/lib_$BASE.so (default head) vs in-tree, two rounds
#   kb_env   tools/kbench.py once per environment setting in $KB_ENVS ("A=1 B=2;A=0", ';'-separated),
#            on $KB_ARGS (default: 2048 pan frames), two rounds
#   ba       tools/babench.py 40 on the in-tree library, three runs
#   ba_env   tools/babench.py 40 once per setting in $BA_ENVS (as kb_env), $BA_ROUNDS rounds (2); ba_timing: one
#            call's host-side phase times (ORBBA_DEBUG_TIMING=1)
#   kb_sweep tools/kbench.py on pan frames at 64 .. 2048 frames per launch (per-frame stage times)
#   stereo   tests/test_stereo_gpu.py      batests  tests/test_ba_gpu.py + tests/test_cpp_dropin_gpu.py
#   pyt      pytest on $PYT_FILES (-m gpu -x -q)
#   ba_prof  rocprofv3 kernel stats of tools/babench.py 20, once per setting in $BA_ENVS (per-kernel averages)
#   pmc_pan | pmc_tex   instruction counters (tools/pmc_groups_inst.txt) on 1024 pan / textured frames, and the
#            per-cell / per-wavefront counts (tools/pmc_percell.py) -> gpurun_out/pmci_{pan,textured}/
#
# Example: gpurun -- 'bash tools/gpu_round.sh tests smoke bench'
#          gpurun -- 'KB_ENVS="ORBX_FAST_SPEC=8;ORBX_FAST_SPEC=-1" bash tools/gpu_round.sh kb_env'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYT="python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread"
for step in "$@"; do
  case $step in
  tests)
    timeout -k 10 900 $PYT tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 2; }
    tail -2 gpurun_out/pytest_gpu.log ;;
  xtests)
    timeout -k 10 600 $PYT tests/test_extractor_gpu.py tests/test_cpp_dropin_gpu.py tests/test_matcher_gpu.py \
      tests/test_compat_gpu.py -m gpu -x -q > gpurun_out/pytest_x.log 2>&1 || { tail -30 gpurun_out/pytest_x.log; exit 2; }
    tail -2 gpurun_out/pytest_x.log ;;
  pjk1)
    ORBSLAM2_AMD_LIB=$PWD/tools/diag/liborbslam2_amd_pjk1.so timeout -k 10 300 $PYT tests/test_projection_gpu.py -q \
      > gpurun_out/pytest_pjk1.log 2>&1 || { tail -20 gpurun_out/pytest_pjk1.log; exit 2; }
    tail -1 gpurun_out/pytest_pjk1.log ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
    tail -1 gpurun_out/smoke.log ;;
  det)
    timeout -k 10 300 python tools/diag/desc_determinism.py > gpurun_out/det.log 2>&1 || { tail -20 gpurun_out/det.log; exit 4; }
    tail -3 gpurun_out/det.log ;;
  bench)
    timeout -k 10 900 python -u bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 7; }
    grep '^{' gpurun_out/bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step']); print(json.dumps(r.get('summary')))" ;;
  ba)
    for i in 1 2 3; do
      timeout -k 10 60 python tools/babench.py 40 > gpurun_out/babench.log 2>&1 || { tail gpurun_out/babench.log; exit 5; }
      grep LocalBA gpurun_out/babench.log
    done ;;
  ba_env)
    IFS=';' read -ra envs <<< "${BA_ENVS:-}"
    for i in $(seq 1 ${BA_ROUNDS:-2}); do
      for e in "${envs[@]}"; do
        env $e timeout -k 10 60 python tools/babench.py 40 > gpurun_out/babench.log 2>&1 || { tail gpurun_out/babench.log; exit 5; }
        grep LocalBA gpurun_out/babench.log | sed "s|^|[$e] |"
      done
    done ;;
  ba_timing)
    ORBBA_DEBUG_TIMING=1 timeout -k 10 60 python tools/babench.py 2 > gpurun_out/ba_timing.log 2>&1 || { tail gpurun_out/ba_timing.log; exit 5; }
    tail -14 gpurun_out/ba_timing.log ;;
  kb_sweep)
    for n in 64 128 256 512 2048; do
      timeout -k 10 120 python tools/kbench.py --frames $n --iters 10 --pan > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/[$n frames] /" gpurun_out/kb.log | tail -1
    done ;;
  batests)
    timeout -k 10 300 $PYT tests/test_ba_gpu.py tests/test_cpp_dropin_gpu.py -q > gpurun_out/pytest_ba.log 2>&1 || { tail -30 gpurun_out/pytest_ba.log; exit 2; }
    tail -2 gpurun_out/pytest_ba.log ;;
  ba_prof)
    IFS=';' read -ra envs <<< "${BA_ENVS:-X=0}"
    k=0
    for e in "${envs[@]}"; do
      k=$((k + 1))
      env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ba_prof$k -o ba -- \
        python3 tools/babench.py 20 > gpurun_out/ba_prof$k.log 2>&1 || { tail gpurun_out/ba_prof$k.log; exit 5; }
      echo "[$e] $(grep LocalBA gpurun_out/ba_prof$k.log)"
      python3 -c "import csv; [print('   %-40s %5s %8.2f us' % (x['Name'].split('(')[0][-40:], x['Calls'], float(x['AverageNs']) / 1e3)) for x in list(csv.DictReader(open('gpurun_out/ba_prof$k/ba_kernel_stats.csv')))[:6]]"
    done ;;
  pyt)
    timeout -k 10 600 $PYT $PYT_FILES -m gpu -x -q > gpurun_out/pytest_pyt.log 2>&1 || { tail -30 gpurun_out/pytest_pyt.log; exit 2; }
    tail -2 gpurun_out/pytest_pyt.log ;;
  stereo)
    timeout -k 10 300 $PYT tests/test_stereo_gpu.py -q > gpurun_out/pytest_stereo.log 2>&1 || { tail -30 gpurun_out/pytest_stereo.log; exit 2; }
    tail -2 gpurun_out/pytest_stereo.log ;;
  ba_ab)
    for i in 1 2 3; do
      ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_${BASE:-head}.so timeout -k 10 60 python tools/babench.py 40 > gpurun_out/babench.log 2>&1 || exit 5
      grep LocalBA gpurun_out/babench.log | sed "s/^/base: /"
      timeout -k 10 60 python tools/babench.py 40 > gpurun_out/babench.log 2>&1 || exit 6
      grep LocalBA gpurun_out/babench.log | sed "s/^/new:  /"
    done ;;
  kb_pan|kb_tex)
    args="--frames 2048 --iters 5 --pan"; [ $step = kb_tex ] && args="--frames 1024 --iters 5 --textured"
    for i in 1 2; do
      ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_${BASE:-head}.so timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$step base: /" gpurun_out/kb.log | tail -1
      timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 9; }
      sed "s/^/$step new:  /" gpurun_out/kb.log | tail -1
    done ;;
  kb_env)
    IFS=';' read -ra envs <<< "${KB_ENVS:-}"
    for i in 1 2; do
      for e in "${envs[@]}"; do
        env $e timeout -k 10 120 python tools/kbench.py ${KB_ARGS:---frames 2048 --iters 5 --pan} > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
        sed "s|^|[$e] |" gpurun_out/kb.log | tail -1
      done
    done ;;
  pmc_pan|pmc_tex)
    w=pan; [ $step = pmc_tex ] && w=textured
    PMC_GROUPS=tools/pmc_groups_inst.txt bash tools/gpu_pmc.sh pmci_$w --$w --frames 1024 > gpurun_out/pmci_$w.log 2>&1 || { tail gpurun_out/pmci_$w.log; exit 10; }
    python3 tools/pmc_percell.py gpurun_out/pmci_$w 1024 | tee gpurun_out/pmci_$w/percell.txt ;;
  *) echo "unknown step $step"; exit 1 ;;
  esac
done
echo "session done"
