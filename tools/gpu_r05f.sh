#!/bin/bash
# round 5: module/rs.h host-pointer pipeline sweep (threads, chunk, zero copy) with the stage trace
set -o pipefail
OUT=gpurun_out/${1:-r05f}; mkdir -p $OUT
source tools/gpu_step.sh
step wire_tests 300 python -u -m pytest tests/test_gpu_wire.py -x -q --timeout 120 --timeout-method thread -k "wave64 or row_tails"
export QFEC_RS_TRACE=1
for th in 16 8 4; do
  for ch in 0 300 3000; do
    step rs_t${th}_c${ch} 200 python tools/rs_abi_rate.py --reps 2 --threads $th --chunk $ch
  done
done
step rs_t16_zc0 200 python tools/rs_abi_rate.py --reps 2 --threads 16 --zero-copy 0
python3 - <<'PY' > $OUT/memcpy.txt 2>&1
import time, numpy as np, torch, threading
a = np.random.default_rng(0).integers(0, 256, 1 << 30, dtype=np.uint8)
p = torch.empty(1 << 30, dtype=torch.uint8).pin_memory().numpy()
q = np.empty(1 << 30, np.uint8)
for dst, name in ((p, "pinned"), (q, "pageable")):
    for nt in (1, 4, 8, 16):
        def job(i):
            n = (1 << 30) // nt
            np.copyto(dst[i * n:(i + 1) * n], a[i * n:(i + 1) * n])
        t0 = time.perf_counter()
        ths = [threading.Thread(target=job, args=(i,)) for i in range(nt)]
        [t.start() for t in ths]; [t.join() for t in ths]
        dt = time.perf_counter() - t0
        print(f"copy 1 GiB pageable -> {name}, {nt} threads: {1 / dt:.1f} GiB/s")
PY
cat $OUT/memcpy.txt
grep -h "value\|\[qfec\]" $OUT/rs_*.log | cut -c1-220
