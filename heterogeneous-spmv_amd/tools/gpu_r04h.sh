#!/bin/bash
# GPU-box pass (round 4 h): the driver's N > 1 default workload (C4, strong
# scaling) through bench.py's multi-rank path, rehearsed as 2 ranks on the
# one GPU with gloo exchanges (RCCL allows one rank per device); checks the
# strong_scaling block end to end.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04h; mkdir -p $O; cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --backend gloo --same-device --steps 50 --warmup 5 \
  > $O/bench_n2_c4_gloo.log 2> $O/bench_n2_c4_gloo.err
rc=$?; echo "rc=$rc"; tail -c 3000 $O/bench_n2_c4_gloo.log; tail -5 $O/bench_n2_c4_gloo.err
