cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ts && \
timeout -k 10 300 python -u tools/two_stream.py --batch 64 --streams 1 1 > gpurun_out/ts/b64.log 2>&1 && \
timeout -k 10 300 python -u tools/two_stream.py --batch 128 --streams 2 1 2 > gpurun_out/ts/b128.log 2>&1
