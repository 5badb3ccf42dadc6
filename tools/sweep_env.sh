#!/bin/bash
# Run bench.py once per value of an environment knob; print the key numbers.
#   bash tools/sweep_env.sh VAR "v1 v2 ..." [bench args]
VAR=$1; VALS=$2; shift 2
for v in $VALS; do
  r=$(env $VAR=$v timeout -k 10 300 python bench.py --no-cpu "$@" 2>/dev/null) || { echo "$VAR=$v failed"; exit 1; }
  python3 -c "
import json,sys; d=json.loads(sys.argv[1]); r=d['roofline']; o=d['roofline_other']
print('$VAR=$v value=%.0f GiB/s  %s %.0f GB/s (%.1f%%)  %s %.0f GB/s (%.1f%%) verified=%s' % (d['value'], r['kernel'], r['achieved'], 100*r['frac'], o['kernel'], o['achieved'], 100*o['frac'], d['verified']))" "$r"
done
