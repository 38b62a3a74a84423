set -u
SNNFLOW_UNET_NSTAGE_DGRAD=333 SNNFLOW_UNET_NSTAGE_CONV=3333 timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/unet_ns3_tests.log 2>&1 || { tail -30 gpurun_out/unet_ns3_tests.log; exit 3; }
tail -2 gpurun_out/unet_ns3_tests.log
AB="X=0 SNNFLOW_UNET_NSTAGE_DGRAD=333 SNNFLOW_UNET_NSTAGE_CONV=2333 SNNFLOW_UNET_NSTAGE_CONV=2233 SNNFLOW_UNET_NSTAGE_CONV=2244" PAT="M32 K160|M512 K512|M288|M160 K32|M64 K288" bash tools/gpu_r6_unet_ab.sh
