set -e
mkdir -p gpurun_out/envstep
for t in CUT MIN_CUT MIN_COVER MAX_IND_SET MAX_CLIQUE MIN_DOM_SET; do
  timeout -k 10 120 python bench.py --workload envstep --target $t --steps 50 --warmup 5 > gpurun_out/envstep/$t.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/envstep/prof_mincover -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload envstep --target MIN_COVER --steps 50 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/envstep/prof_mincover.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/envstep/prof_cut -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload envstep --target CUT --steps 50 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/envstep/prof_cut.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/envstep/fetch_mincover -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload envstep --target MIN_COVER --steps 20 --warmup 2 > /dev/null
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/envstep/write_mincover -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload envstep --target MIN_COVER --steps 20 --warmup 2 > /dev/null
echo done
