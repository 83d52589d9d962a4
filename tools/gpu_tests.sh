# GPU test run: the -m gpu tests of the given files (default: all), then smoke().  TAG names gpurun_out/<TAG>.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-t}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest ${@:-tests} -m gpu -x -v -s --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
