set -u
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py -m gpu -x -q -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/unet_tests.log 2>&1 || { grep -E "^E |Error|error" gpurun_out/unet_tests.log | head -30; tail -5 gpurun_out/unet_tests.log; exit 3; }
tail -1 gpurun_out/unet_tests.log
AB="X=0 SNNFLOW_UNET_DGRAD8=0" PAT="dgrad" bash tools/gpu_r6_unet_ab.sh || exit 4
