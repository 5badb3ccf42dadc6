#!/bin/bash
# The one parametrised GPU-box runner (round 6; replaces the per-run tools/gpu_r0*.sh scripts).
#   gpurun --timeout 1200 -- bash tools/gpu_run.sh TAG 'STEP ARGS...' ['STEP ARGS...' ...]
# Every step runs under its own time limit (tools/gpu_step.sh) and writes gpurun_out/TAG/<name>.log;
# a timeout, abort or crash ends the call there.  Steps:
#   tests EXPR            python -m pytest tests -m gpu -k EXPR (EXPR "all": the whole GPU suite)
#   ab K M B G ONLY [ARGS...]
#                         tools/ab.py interleaved A/B (ONLY: comma-separated variant prefixes)
#   bench [ARGS...]       bench.py -> TAG/bench.json (stderr TAG/bench.err)
#   kstats [ARGS...]      rocprofv3 --kernel-trace --stats over bench.py --no-cpu --no-host --no-side -> TAG/prof/,
#                         summary TAG/kernel_stats.csv
#   pmc NAME K M B G [ARGS...]
#                         tools/pmc_traffic.py (separate --pmc passes per counter group) -> TAG/traffic_NAME.json
#   sq NAME SCRIPT [ARGS...]
#                         SQ counters per kernel (two --pmc passes over python SCRIPT) -> TAG/NAME_sq_summary.txt
#   smoke                 __graft_entry__.smoke()
#   bench2                bench.py --gpus 2 with gloo (the launcher's two ranks share the one GPU) -> TAG/bench_g2.json
#   wirestats             rocprofv3 kernel stats of the datagram kernels at the wire leg's shapes -> TAG/wire_kernel_stats.csv
#   merge_traffic         the TAG/traffic_*.json entries of earlier pmc steps into profiles/traffic.json (on the box,
#                         so a later bench step reads them; copy it back from TAG/traffic.json)
#   closing               the end-of-round pass: tests all, smoke, pmc h / c4 / wire, merge_traffic, bench, kstats,
#                         wirestats, bench2 (the steps of the former tools/gpu_full.sh + gpu_final.sh)
#   py NAME SECS ARGS...  any python command (tools/*.py), log TAG/NAME.log
#   pyenv NAME SECS VAR=VALUE ARGS...  the same with one environment variable set
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
source tools/gpu_step.sh
n=0
specs=()
for spec in "$@"; do
  if [ "$spec" = closing ]; then
    specs+=("tests all" smoke "pmc h 10 3 1024 100000" "pmc c4 16 4 1400 250000 --workload config4"
            "pmc wire 10 3 1024 100000 --workload wire" merge_traffic bench kstats wirestats bench2)
  else
    specs+=("$spec")
  fi
done
for spec in "${specs[@]}"; do
  n=$((n + 1))
  set -- $spec
  what=$1; shift
  case $what in
    tests)
      expr="$*"
      if [ "$expr" = all ]; then
        step tests_all 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
      else
        step tests_$n 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$expr"
      fi ;;
    ab)
      k=$1 m=$2 b=$3 g=$4 only=$5; shift 5
      step ab_${k}_${m}_${b}_${g}_$n 420 python -u tools/ab.py --k $k --m $m --block $b --groups $g --only "$only" "$@"
      tail -30 $OUT/ab_${k}_${m}_${b}_${g}_$n.log ;;
    bench)
      echo "== bench"
      timeout -k 10 400 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
      rc=$?; echo "   rc=$rc"; cat $OUT/bench.json
      if [ $rc -ne 0 ]; then tail -30 $OUT/bench.err; exit $rc; fi ;;
    kstats)
      echo "== rocprofv3 kernel stats"
      # only the timed step's launches and config 4's (the host / per-call / side legs launch the same
      # kernels at other sizes), so each kernel's average is the one bench.py reports
      timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
        python3 bench.py --no-cpu --no-host --no-side "$@" > $OUT/kstats.log 2>&1
      rc=$?; echo "   rc=$rc"; tail -3 $OUT/kstats.log
      if [ $rc -ne 0 ]; then exit $rc; fi
      f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1)
      [ -n "$f" ] && cp "$f" $OUT/kernel_stats.csv && cut -d, -f1-5 $OUT/kernel_stats.csv | head -12 ;;
    pmc)
      name=$1 k=$2 m=$3 b=$4 g=$5; shift 5
      step pmc_$name 900 python -u tools/pmc_traffic.py --out $OUT/pmc_$name --json $OUT/traffic_$name.json \
        --tag "$TAG" --k $k --m $m --block $b --groups $g "$@"
      ;;
    sq)
      # SQ counters (issue / wait split, instruction mix) per kernel: two --pmc passes over one
      # python command (a script path relative to the repo, then its arguments)
      name=$1 script=$2; shift 2
      R=$(pwd); j=0
      for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
                 "SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU"; do
        j=$((j + 1))
        echo "== sq $name pass $j"
        (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $set --output-format csv -d $R/$OUT/${name}_sq$j -o p -- \
          python3 $R/$script "$@" > $R/$OUT/${name}_sq$j.log 2>&1)
        rc=$?; echo "   rc=$rc"
        if [ $rc -ne 0 ]; then tail -5 $OUT/${name}_sq$j.log; exit $rc; fi
      done
      python3 tools/sq_summary.py $OUT/${name}_sq1 $OUT/${name}_sq2 > $OUT/${name}_sq_summary.txt
      cat $OUT/${name}_sq_summary.txt ;;
    bench2)
      echo "== bench --gpus 2 (gloo)"
      QFEC_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 20 --no-cpu > $OUT/bench_g2.json 2> $OUT/bench_g2.err
      rc=$?; echo "   rc=$rc"; cut -c1-400 $OUT/bench_g2.json
      if [ $rc -ne 0 ]; then tail -20 $OUT/bench_g2.err; exit $rc; fi ;;
    wirestats)
      echo "== rocprofv3 kernel stats, datagram kernels (tools/side_legs.py)"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_wire -o wire -- \
        python3 tools/side_legs.py --steps 100 > $OUT/side_prof.json 2> $OUT/side_prof.err
      rc=$?; echo "   rc=$rc"
      if [ $rc -ne 0 ]; then tail -20 $OUT/side_prof.err; exit $rc; fi
      f=$(find $OUT/prof_wire -name '*kernel_stats.csv' | head -1)
      [ -n "$f" ] && cp "$f" $OUT/wire_kernel_stats.csv && cut -d, -f1-5 $OUT/wire_kernel_stats.csv | cut -c1-160 | head -10 ;;
    merge_traffic)
      python3 - "$OUT" <<'PY' || exit 11
import glob, json, os, sys
out = sys.argv[1]
main = json.load(open("profiles/traffic.json"))
for f in sorted(glob.glob(os.path.join(out, "traffic_*.json"))):
    name = os.path.basename(f)[len("traffic_"):-len(".json")]
    for key, ent in json.load(open(f)).items():
        if ent.get("run") == os.path.basename(out):
            ent["csv"] = f"profiles/{os.path.basename(out)}/pmc/{name}"
            main[key] = ent
            print("merged", key, "from", f)
json.dump(main, open("profiles/traffic.json", "w"), indent=1)
json.dump(main, open(os.path.join(out, "traffic.json"), "w"), indent=1)
PY
      ;;
    smoke)
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    py)
      name=$1 secs=$2; shift 2
      step $name $secs python -u "$@" ;;
    pyenv)
      # pyenv NAME SECS VAR=VALUE SCRIPT [ARGS...]: the same with one environment variable set
      name=$1 secs=$2 var=$3; shift 3
      step $name $secs env "$var" python -u "$@" ;;
    *)
      echo "unknown step '$what'"; exit 2 ;;
  esac
done
echo "== done $TAG"
