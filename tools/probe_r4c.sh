#!/bin/bash
# dev: conv3w at the bench batch, stamped builds (cycles, clock, per-unit periods of the second
# tile): shipped kernel vs ablations (a1 no mid-unit barrier, a3 no fragment reads, a4 no DMA after
# the prologue, nost no output stores) and non-temporal epilogue stores (snt)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/probe && {
for r in 1 2; do
  for v in bin bin_a1 bin_a3 bin_a4 bin_nost bin_snt; do
    echo "== $v rep $r" && timeout -k 5 60 tools/conv3w_probe_$v 130 46 82 128 128 20 1 || exit 1
  done
done
for v in bin bin_a3 bin_a4 bin_nost; do
  echo "== $v zero operands" && timeout -k 5 60 tools/conv3w_probe_$v 130 46 82 128 128 20 1 1 || exit 1
done ; } > gpurun_out/probe/${1:-r4c}.log 2>&1
