cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/tl -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/tl.log 2>&1
