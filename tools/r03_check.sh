#!/bin/bash
# GPU box: the driver's round-end sequence rehearsed on the committed tree -- the -m gpu suite, smoke(), then the
# default bench line (with the CPU baselines) and the configs[4] / configs[3] lines.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/chk"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$ROOT/gpurun_out/chk/gputests.log" 2>&1
rc=$?; tail -3 "$ROOT/gpurun_out/chk/gputests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$ROOT/gpurun_out/chk/smoke.log" 2>&1 || { tail -5 "$ROOT/gpurun_out/chk/smoke.log"; exit 4; }
tail -1 "$ROOT/gpurun_out/chk/smoke.log"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > "$ROOT/gpurun_out/chk/bench.json" 2> "$ROOT/gpurun_out/chk/bench.err" || exit 5
python3 -c "import json; d=json.loads(open('$ROOT/gpurun_out/chk/bench.json').read().strip().splitlines()[-1]); print('train', round(d['value']), round(d['ms_per_step'],3), d['roofline']['frac'], d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
timeout -k 10 300 python -u bench.py --workload gset --steps 20 --warmup 3 > "$ROOT/gpurun_out/chk/gset.json" 2>/dev/null || exit 6
python3 -c "import json; d=json.loads(open('$ROOT/gpurun_out/chk/gset.json').read().strip().splitlines()[-1]); print('gset', round(d['value']), round(d['ms_per_step'],3))"
