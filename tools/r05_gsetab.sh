#!/bin/bash
# GPU box: configs[4] (gset) per library build: the shared-graph parity test, the bench line (twice, interleaved),
# then FETCH_SIZE / WRITE_SIZE passes (one counter set per rocprofv3 run) summed over the forward's kernels.
# usage: bash tools/r05_gsetab.sh <tag> <lib suffix|product> ...
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
libpath() { [ "$1" = product ] && echo "$ROOT/eco-dqn_amd/eco_hip/libecohip.so" || echo "$ROOT/eco-dqn_amd/eco_hip/libecohip_$1.so"; }
for v in "$@"; do
  ECO_HIP_LIB=$(libpath $v) timeout -k 10 300 python -u -m pytest tests/test_parity_benched_batches_gpu.py -m gpu -k gset -x -q \
    --timeout 240 --timeout-method thread -p no:cacheprovider > "$OUT/test_$v.log" 2>&1 || { echo "test $v failed"; tail -5 "$OUT/test_$v.log"; exit 3; }
  echo "test $v ok"
done
for rep in 1 2; do
  for v in "$@"; do
    ECO_HIP_LIB=$(libpath $v) timeout -k 10 300 python -u bench.py --workload gset --steps 5 --warmup 2 --no-cpu-baseline \
      > "$OUT/gset_${v}_$rep.json" 2> "$OUT/gset_${v}_$rep.err" || { tail -5 "$OUT/gset_${v}_$rep.err"; exit 4; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['ms_per_step'],3))" "$OUT/gset_${v}_$rep.json" "$v r$rep"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  for C in FETCH_SIZE WRITE_SIZE; do
    ECO_HIP_LIB=$(libpath $v) timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${v}_$C" -o run -- \
      python3 "$ROOT/bench.py" --workload gset --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_${v}_$C.log" 2>&1 || { echo "pmc $v $C failed"; exit 5; }
  done
  python3 - "$OUT" "$v" <<'PY'
import csv, glob, sys, collections
out, v = sys.argv[1], sys.argv[2]
tot = collections.Counter(); n = collections.Counter()
for C in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{out}/pmc_{v}_{C}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            if "shared_" in k:
                tot[C] += float(row["Counter_Value"])
                if C == "FETCH_SIZE": n[k.split("(")[0]] += 1
print(v, {c: round(t / 1e6, 3) for c, t in tot.items()}, "(counter units x1e6, 3 forwards incl. warmup)", dict(n))
PY
done
