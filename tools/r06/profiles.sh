#!/bin/bash
# GPU box, round 6: the profiles behind the bench line and the configs lines.
#   1) default train bench (configs[2]): kernel trace + stats, FETCH_SIZE pass, WRITE_SIZE pass (tools/run_profile.sh)
#   2) configs[3] (BA-500 train), configs[4] (G22-like), configs[1] (ER-20) and the env-step sub-bench under
#      rocprofv3 --kernel-trace --stats
#   3) SQ counters of the dense ER-200 M=2048 forward / training forward / backward (tools/pmc_dense.sh)
# Each GPU step under its own time limit; the script stops at the first failure.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06final}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
bash "$ROOT/tools/run_profile.sh" "$TAG" > "$OUT/run_profile.log" 2>&1 || { tail -5 "$OUT/run_profile.log"; exit 3; }
python3 "$ROOT/tools/pmc_summary.py" "$ROOT/gpurun_out/prof_$TAG" "$OUT/train" || exit 4
cd /tmp && export TMPDIR=/tmp
for w in ba500 gset er20 envstep; do
  case $w in
    ba500) args="--graph BA --n 500 --steps 4 --warmup 2 --no-cpu-baseline";;
    gset) args="--workload gset --steps 20 --warmup 3";;
    er20) args="--workload er20 --steps 40 --warmup 5";;
    envstep) args="--workload envstep --steps 100 --warmup 5";;
  esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/$w" -o run -- \
    python3 "$ROOT/bench.py" $args > "$OUT/$w.json" 2> "$OUT/$w.err" || { tail -5 "$OUT/$w.err"; exit 5; }
  python3 -c "import json; d=json.loads(open('$OUT/$w.json').read().strip().splitlines()[-1]); print('$w', round(d['value']), 'ms/step', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4))"
done
cd "$ROOT"
bash "$ROOT/tools/pmc_dense.sh" > /dev/null 2>&1 || { echo "pmc_dense failed"; exit 6; }
python3 "$ROOT/tools/pmc_sq_summary.py" "$ROOT/gpurun_out/pmc_dense.txt" "$OUT/train/pmc_sq_dense.json" || exit 7
echo "profiles done"
