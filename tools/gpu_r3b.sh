cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3b
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 120 --timeout-method thread -k "multiscale or upsampling" > gpurun_out/r3b/pytest.log 2>&1 || exit 1
bash tools/pmc_round.sh pmc_body135 --config body135
