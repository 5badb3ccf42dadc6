set -o pipefail
O=gpurun_out/r02zi; mkdir -p $O
for al in 16 64 16 64; do
  timeout -k 10 120 python tools/wire_ab.py --unpack --align $al --variants base --rounds 8 >> $O/unpack_align.txt 2>&1 || exit 2
  timeout -k 10 120 python tools/wire_ab.py --align $al --variants base --rounds 8 >> $O/pack_align.txt 2>&1 || exit 3
done
for al in 16 64; do
  timeout -k 10 120 python tools/wire_ab.py --unpack --size 1400 --align $al --variants base --rounds 8 >> $O/unpack_align.txt 2>&1 || exit 2
  timeout -k 10 120 python tools/wire_ab.py --size 1400 --align $al --variants base --rounds 8 >> $O/pack_align.txt 2>&1 || exit 3
done
grep -v amdgpu.ids $O/unpack_align.txt; grep -v amdgpu.ids $O/pack_align.txt
