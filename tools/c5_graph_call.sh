set -u
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/c5g
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "spectral_null or c5 or graph or host_io or label_difference" > gpurun_out/c5g/tests.log 2>&1 || { tail -40 gpurun_out/c5g/tests.log; exit 1; }
tail -3 gpurun_out/c5g/tests.log
timeout -k 10 120 python3 tools/c5_graph_trace.py > gpurun_out/c5g/plain.json 2> gpurun_out/c5g/plain.err || { tail -20 gpurun_out/c5g/plain.err; exit 2; }
cat gpurun_out/c5g/plain.json
cd /tmp && export TMPDIR=/tmp
C5_STEPS=200 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d $R/gpurun_out/c5g/prof -o c5g --output-format csv -- python3 $R/tools/c5_graph_trace.py > $R/gpurun_out/c5g/prof.log 2>&1 || { tail -20 $R/gpurun_out/c5g/prof.log; exit 3; }
tail -2 $R/gpurun_out/c5g/prof.log
find $R/gpurun_out/c5g/prof -name "*.csv" | head
