#!/bin/bash
# Launcher readiness on the GPU box: box topology as sysfs shows it, the launch tests, the
# default bench line (NUMA / CPU-share fields), and a 2-rank gloo rehearsal.
#   gpurun --timeout 900 -- bash tools/gpu_launch.sh TAG
set -o pipefail
TAG=${1:-launch}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
{
  echo "== env"; env | grep -E "VISIBLE|ROCR|OMP_NUM|HIP_" ; echo "nproc $(nproc)"
  python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
  for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu/cpu.cfs_quota_us /sys/fs/cgroup/cpu/cpu.cfs_period_us; do [ -r $f ] && echo "$f: $(cat $f)"; done
  echo "== kfd nodes"; for d in /sys/class/kfd/kfd/topology/nodes/*; do echo "$d: $(grep -E 'gfx_target_version|location_id|domain|unique_id|simd_count' $d/properties | tr '\n' ' ')"; done
  echo "== topology.py"; python -c "
from quicknet_amd import topology as T
print(T.gpu_count()); print(T.visible_gpus()); p=T.gpu_numa(0); print(p and {k:(sorted(v)[:4]+['...',len(v)] if k=='cpus' else v) for k,v in p.items()}); print(T.cpu_share())"
} > $OUT/topology.txt 2>&1
cat $OUT/topology.txt | head -40
echo "== launch tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_launch.py -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_launch.log 2>&1 || { tail -40 $OUT/pytest_launch.log; exit 2; }
grep -E "PASS|FAIL|launch-check|numa:" $OUT/pytest_launch.log
echo "== bench (N=1)"
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 3; }
python -c "
import json; d=[json.loads(l) for l in open('$OUT/bench.json') if l.startswith('{')][-1]
print({k: d[k] for k in ('value','verified','host_cpus','per_rank_numa','numa_binding_rank0','process_group')})
print('cpu_mt', d['cpu_baseline_threads']); print('ref check', d['host_to_host_mixed'].get('reference_check'))"
echo "== bench --gpus 2 (gloo rehearsal)"
QFEC_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --no-cpu > $OUT/bench_g2.json 2> $OUT/bench_g2.err || { tail -30 $OUT/bench_g2.err; exit 4; }
python -c "
import json; d=[json.loads(l) for l in open('$OUT/bench_g2.json') if l.startswith('{')][-1]
print({k: d[k] for k in ('value','verified','n_gpus','per_rank_numa','numa_binding_rank0','process_group')})"
