#!/bin/bash
# Static wave priorities (s_setprio 1), interleaved A/B against the product
# library: prioA = config 2's recompute waves, config 4's backward rows,
# config 3's partners; prioB = config 2's partners, config 4's forward rows,
# config 3's filters.  Then chain_estep16_kernel's per-wave phase stamps in
# proper mode (em) and general mode (estep), and the em split point H.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04y; mkdir -p $O
L=nip_amd/_lib/ab
for wl in estep em fb config3; do
  bash profiles/r04/ab_tests.sh r04y/$wl $wl "" $L/prioA.so $L/prioB.so || exit 1
done
for w in em estep; do
  timeout -k 10 300 env NIPAMD_LIB=$PWD/$L/stamps.so NIPAMD_PHASE_TIMES=1 python bench.py --workload $w \
    --steps 1 --warmup 1 --no-secondary --no-cpu-baseline --no-check > $O/stamps_$w.txt 2>&1 || exit 1
done
for h in 40 50 60; do
  timeout -k 10 300 env NIPAMD_LIB=$PWD/$L/diag.so NIPAMD_ESTEP_H=$h python bench.py --workload em \
    --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-check > $O/h${h}_em.txt 2>&1 || exit 1
done
echo done
