#!/bin/bash
# GPU-box pass: the host AddressSanitizer + UBSan build (make asan, built on
# the CPU beforehand) drives spmv-csr / spmv-csrk over the golden matrices
# and generated power-law / banded / stencil ones, with every kernel and
# CSR-3 plan, so the host planner (tables, x dictionaries, csort blocks, band-k
# maps, readers) runs instrumented at real sizes.  Device code is not
# instrumented.  The first sanitizer report or failed check ends the pass with
# that status; logs under gpurun_out/TAG_asan/.
# Usage (from the repo root): bash heterogeneous-spmv_amd/tools/host_asan.sh [TAG]
set -o pipefail
TAG=${1:-asan}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/${TAG}_asan; mkdir -p $O
B=$R/heterogeneous-spmv_amd/build/asan
G=$R/tests/golden
D=$(mktemp -d)  # generated inputs (kept out of gpurun_out/)
trap 'rm -rf $D' EXIT
# verify_asan_link_order=0: a preloaded library may precede the runtime
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:verify_asan_link_order=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
timeout -k 10 300 python3 - "$D" <<'EOF' || exit $?
import sys
sys.path.insert(0, "heterogeneous-spmv_amd")
import numpy as np
from hspmv import gen
o = sys.argv[1]
gen.write_csr_text(f"{o}/powerlaw.csr", gen.powerlaw(200_000, seed=5, dtype=np.float64))
gen.write_csr_text(f"{o}/banded.csr", gen.banded(300_000, per_row=12, half=40, seed=3))
gen.write_csr_text(f"{o}/stencil.csr", gen.stencil27(40, seed=7))
EOF
n=0
step() {  # step LOGNAME CMD...
  local name=$1; shift
  n=$((n + 1))
  timeout -k 10 180 "$@" > $O/$name.log 2>&1; local rc=$?
  if [ $rc -ne 0 ] || grep -q "AddressSanitizer\|runtime error:" $O/$name.log; then
    echo "FAIL $name rc=$rc"; tail -30 $O/$name.log; exit $(( rc ? rc : 1 ))
  fi
}
for f in $G/*.csr $D/powerlaw.csr $D/banded.csr $D/stencil.csr; do
  b=$(basename $f .csr)
  for k in auto stream vector:8 csr3 csort; do
    step "csr_${b}_${k/:/}" $B/spmv-csr $f 3 --kernel $k --x rand:1
  done
  step "csr_${b}_f32" $B/spmv-csr $f 3 --dtype f32 --x rand:1
  step "csr_${b}_det" $B/spmv-csr $f 3 --deterministic --x rand:1
  step "csr_${b}_repro" $B/spmv-csr $f 3 --kernel csort --reproducible --x rand:1
  step "csr_${b}_repro_f32" $B/spmv-csr $f 3 --kernel csort --reproducible --dtype f32 --x rand:1
  step "csr_${b}_serial" $B/spmv-csr $f 3 --serial --x rand:1
  step "csr_${b}_serial_f32" $B/spmv-csr $f 3 --serial --dtype f32 --x rand:1
done
for f in $G/*.csr3; do
  b=$(basename $f .csr3)
  step "csrk_${b}_serial" $B/spmv-csrk $f 3 --serial --plan ssr --x rand:2
done
for f in $G/*.csr3; do
  b=$(basename $f .csr3)
  for p in aligned packed ssr; do
    step "csrk_${b}_${p}" $B/spmv-csrk $f 3 --plan $p --x rand:2
  done
done
for f in $G/powerlaw1500.csr $D/stencil.csr $D/banded.csr; do
  b=$(basename $f .csr)
  step "csrk_${b}_bandk" $B/spmv-csrk $f 3 20 10 --x rand:3
  step "csrk_${b}_csr2" $B/spmv-csrk $f 3 8 --x rand:3
  step "csrk_${b}_bandk_ssr" $B/spmv-csrk $f 3 20 10 --plan ssr --x rand:3
done
for f in $O/*.log; do echo "$(basename $f .log): $(grep -E '^(Kernel|Check):' $f | tr '\n' ' ')"; done > $O/summary.txt
echo "host_asan: $n runs, no sanitizer report"
