#!/bin/bash
# round-4 GPU call: new parity tests (+ the fault-injected variant, expected to fail), the GPU
# suite, smoke, bench.  OUT_TAG=<dir>  STEPS=<env,new,fault,tests,smoke,bench,multi,b135,prof,pmc>
# (pmc: PMC_COMMIT=<sha of the tree> -- the box has no .git)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT_TAG:-r4}
STEPS=${STEPS:-env,new,fault,tests,smoke,bench}
mkdir -p $OUT
run() { case ",$STEPS," in *",$1,"*) return 0;; *) return 1;; esac; }
PYT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
if run env; then
  { nproc; python -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)), 'OMP', os.environ.get('OMP_NUM_THREADS'))"; } > $OUT/env.log 2>&1
fi
if run new; then
  timeout -k 10 500 $PYT -m gpu tests/test_gpu_layers.py "tests/test_gpu_net.py::test_body25_bench_geometry_vs_oracle" tests/test_preprocess.py > $OUT/pytest_new.log 2>&1 || exit 1
fi
if run fault; then
  # the round-3 miscompile reproduced in a dev variant: the per-layer test must FAIL on it
  OPK_LIB_PATH=openpose_amd/variants/libopk_faultpool.so timeout -k 10 300 $PYT -m gpu tests/test_gpu_layers.py > $OUT/pytest_fault_variant.log 2>&1
  rc=$?; echo "exit $rc (1 = test failed as expected)" >> $OUT/pytest_fault_variant.log
  [ $rc -ge 2 ] && exit 1
fi
if run tests; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
fi
if run smoke; then
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
fi
if run bench; then
  timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || exit 1
fi
if run multi; then
  timeout -k 10 300 python -u bench.py --config multiscale --steps 20 > $OUT/bench_multiscale.log 2>&1 || exit 1
fi
if run b135; then
  timeout -k 10 300 python -u bench.py --config body135 > $OUT/bench_body135.log 2>&1 || exit 1
fi
if run prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_prof.log 2>&1 || exit 1
fi
if run nmsab; then   # NMS walk A/B (NMS_WALK variants), post-processing ms per step from the bench line
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pipeline.py -k "nms_walk or multiscale or upsampling or fixture" > $OUT/pytest_nms.log 2>&1 || exit 1
  for i in 1 2; do
    for v in ${NMS_VARIANTS:-0 1 3 4 5 7}; do
      timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --dev NMS_WALK=$v > $OUT/nmsab_b25_w${v}_$i.log 2>&1 || exit 1
      timeout -k 10 200 python -u bench.py --config body135 --steps 20 --no-cpu-baseline --dev NMS_WALK=$v > $OUT/nmsab_b135_w${v}_$i.log 2>&1 || exit 1
    done
  done
fi
if run ab; then   # build A/B: AB_LIBS (variant names; "default" = the product build), interleaved
  for i in 1 2; do
    for v in ${AB_LIBS:-base default}; do
      if [ "$v" = default ]; then L=""; else L="OPK_LIB_PATH=openpose_amd/variants/libopk_$v.so"; fi
      env $L timeout -k 10 200 python -u bench.py --steps 30 --no-cpu-baseline $AB_ARGS > $OUT/ab_${v}_$i.log 2>&1 || exit 1
    done
  done
fi
if run abprof; then   # per-kernel statistics of each A/B build (rocprofv3 kernel trace, 10 steps)
  for v in ${AB_LIBS:-base default}; do
    if [ "$v" = default ]; then export -n OPK_LIB_PATH; unset OPK_LIB_PATH; else export OPK_LIB_PATH=openpose_amd/variants/libopk_$v.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline $AB_ARGS > $OUT/prof_$v.log 2>&1 || exit 1
  done
  unset OPK_LIB_PATH
fi
if run convtests; then
  timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_net.py tests/test_gpu_layers.py > $OUT/pytest_conv.log 2>&1 || exit 1
fi
if run nmsprof; then   # per-kernel statistics of the NMS walk variants (NMS_VARIANTS), body25 + body135
  for v in ${NMS_VARIANTS:-0 8}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/nprof_b135_$v -o run -- python bench.py --config body135 --steps 10 --warmup 2 --no-cpu-baseline --dev NMS_WALK=$v > $OUT/nprof_b135_$v.log 2>&1 || exit 1
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/nprof_b25_$v -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dev NMS_WALK=$v > $OUT/nprof_b25_$v.log 2>&1 || exit 1
  done
fi
if run nmspmc; then   # instruction mix of the NMS walks (body135), one counter pass per variant
  for v in ${NMS_VARIANTS:-0 8}; do
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/npmc_$v -o run -- python bench.py --config body135 --steps 3 --warmup 1 --no-cpu-baseline --dev NMS_WALK=$v > $OUT/npmc_$v.log 2>&1 || exit 1
  done
fi
if run msab; then   # multi-scale (config 4, 4 sources) NMS walk A/B
  for i in 1 2; do
    for v in ${NMS_VARIANTS:-0 8}; do
      timeout -k 10 200 python -u bench.py --config multiscale --steps 15 --no-cpu-baseline --dev NMS_WALK=$v > $OUT/msab_w${v}_$i.log 2>&1 || exit 1
    done
  done
fi
if run pmc; then   # counter passes at this tree (config 2 at the bench batch, config 5 at 64 frames)
  PMC_COMMIT=$PMC_COMMIT bash tools/pmc_round.sh ${OUT_TAG:-r4}/pmc || exit 1
  PMC_COMMIT=$PMC_COMMIT bash tools/pmc_round.sh ${OUT_TAG:-r4}/pmc_body135 --config body135 --batch 64 || exit 1
fi
