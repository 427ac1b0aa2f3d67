cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r2d && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -rA --timeout 120 --timeout-method thread > gpurun_out/r2d/pytest_gpu.log 2>&1 && \
bash tools/pmc_traffic.sh && bash tools/pmc_conv.sh
