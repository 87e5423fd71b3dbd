mkdir -p gpurun_out
PCR_MEANS_G=4 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extractor.py -m gpu -p no:cacheprovider > gpurun_out/t.log 2>&1 || exit 1
PCR_MEANS_G=8 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extractor.py -m gpu -p no:cacheprovider >> gpurun_out/t.log 2>&1 || exit 1
for G in 2 4 8; do for NT in 256 512; do
echo "== G=$G NT=$NT" >> gpurun_out/sp.log
PCR_MEANS_G=$G PCR_PREP_NT=$NT timeout -k 10 100 python -u scripts/stream_probe.py means prep >> gpurun_out/sp.log 2>&1 || exit 1
PCR_MEANS_G=$G PCR_PREP_NT=$NT timeout -k 10 200 python -u scripts/compare_modes.py native1:40 >> gpurun_out/sp.log 2>&1 || exit 1
done; done
