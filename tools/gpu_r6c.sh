mkdir -p gpurun_out/r6c
timeout -k 10 400 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_c5.py tests/test_gpu_queue.py tests/test_gpu_ring.py tests/test_gpu_dense.py -v --timeout 180 --timeout-method thread > gpurun_out/r6c/new_tests.txt 2>&1
rc=$?
tail -30 gpurun_out/r6c/new_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread --deselect tests/test_gpu_timed.py > gpurun_out/r6c/gpu_tests.txt 2>&1
rc2=$?
tail -5 gpurun_out/r6c/gpu_tests.txt
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then exit $rc2; fi
timeout -k 10 300 python bench.py > gpurun_out/r6c/bench.json 2> gpurun_out/r6c/bench.err
tail -c 400 gpurun_out/r6c/bench.err
