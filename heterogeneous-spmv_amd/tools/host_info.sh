# Records the lease's host and GPU configuration into $1 (default
# gpurun_out/host.txt): CPU topology and cgroup quota, and -- for the
# box-to-box spread of C3's fabric traffic -- the GPU's compute and memory
# partition modes, VRAM, clocks, PCIe/xGMI placement (read-only queries).
O=${1:-gpurun_out/host.txt}
mkdir -p "$(dirname "$O")"
{
  echo "== date"; date -u
  echo "== lscpu"; lscpu
  echo "== nproc / cgroup / affinity"; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null
  python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
  env | grep -E '^(OMP|MAX_JOBS|GPU_MAX|HIP_VISIBLE|ROCR_VISIBLE|HSA_)' | sort
  echo "== rocm-smi partitions"; timeout 60 rocm-smi --showcomputepartition --showmemorypartition 2>&1
  echo "== rocm-smi product / bus / vram / clocks"
  timeout 60 rocm-smi --showproductname --showbus --showmeminfo vram --showclocks --showfwinfo 2>&1 | grep -v '^$'
  echo "== amd-smi static"; timeout 60 amd-smi static 2>&1 | head -200
  echo "== amd-smi partition"; timeout 60 amd-smi partition 2>&1 | head -60
  # amdgpu module parameters (mtype_local etc. set the L2 caching mode of
  # local VRAM) and the kernel command line, where readable
  echo "== amdgpu module parameters"
  for f in /sys/module/amdgpu/parameters/*; do [ -r "$f" ] && printf '%s=%s\n' "$(basename $f)" "$(cat $f 2>/dev/null)"; done
  echo "== kernel cmdline"; cat /proc/cmdline 2>/dev/null
  echo "== rocminfo (agent 2)"; timeout 60 rocminfo 2>&1 | grep -E 'Marketing|Compute Unit|Max Clock|Size:|Segment|L2|Cacheline' | head -40
} > "$O" 2>&1
echo "host info -> $O"
B=$(dirname "$0")/../build
if [ -x $B/probes/xcd_map_probe ]; then
  { echo "== workgroup -> XCD mapping (tools/xcd_map_probe.hip)"; timeout -k 5 60 $B/probes/xcd_map_probe 2048 256; timeout -k 5 60 $B/probes/xcd_map_probe 256 1024; } >> "$O" 2>&1
fi
