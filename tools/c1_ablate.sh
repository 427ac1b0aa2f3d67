cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/c1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c1/base -o run -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/c1/base.log 2>&1 && \
for v in 1 2 3; do OPK_LIB_PATH=$GRAFT_REPO_ROOT/openpose_amd/variants/libopk_c1a$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c1/a$v -o run -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/c1/a$v.log 2>&1 || exit 1; done
