mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extractor.py -m gpu -p no:cacheprovider > gpurun_out/t.log 2>&1 || exit 1
timeout -k 10 100 python -u scripts/host_rate.py three_stream native1 native0 > gpurun_out/sp.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/compare_modes.py two_fused:50 three_stream:50 native1:50 native0:50 native1:200 >> gpurun_out/sp.log 2>&1 || exit 1
