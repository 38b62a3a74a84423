set -u
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/unet_tests.log 2>&1 || { tail -30 gpurun_out/unet_tests.log; exit 3; }
tail -1 gpurun_out/unet_tests.log
AB="X=0" PAT="M288|M544|M512 K512|M32 K160" bash tools/gpu_r6_unet_ab.sh || exit 4
bash tools/pmc_unet.sh > gpurun_out/pmc_unet_summary.txt 2>&1; tail -40 gpurun_out/pmc_unet_summary.txt | cut -c1-700
