#!/bin/bash
# GPU-box pass (round 4 g): PMC HBM traffic of the bench workloads c3, c5,
# c5r (separate --pmc passes, gpu_pmc_bench.sh), kernel-trace stats of the
# other configs (gpu_kstats.sh), then the CPU baseline's process-settings A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; T=heterogeneous-spmv_amd/tools
for cfg in c3 c5 c5r; do
  echo "== pmc $cfg"
  timeout -k 10 900 bash $T/gpu_pmc_bench.sh r04g_$cfg "--config $cfg" > gpurun_out/r04g_pmc_$cfg.log 2>&1
  rc=$?; echo "   rc=$rc"; tail -2 gpurun_out/r04g_pmc_$cfg.log | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
done
echo "== kstats"
timeout -k 10 900 bash $T/gpu_kstats.sh r04g "c3 c3:f32 c3h c4 c5 c5r c2" > gpurun_out/r04g_kstats.log 2>&1
rc=$?; echo "   rc=$rc"; [ $rc -ne 0 ] && exit $rc
echo "== cpu A/B"
timeout -k 10 600 python $T/cpu_baseline_ab.py --out gpurun_out/r04g_cpu/cpu_baseline_ab.jsonl --budget 6 --reps 2 > gpurun_out/r04g_cpu_ab.log 2>&1
echo "   rc=$?"
