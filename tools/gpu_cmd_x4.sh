# four mads per asm statement in the reduced-radix products: parity, then A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batch.py tests/test_gpu_ecfft.py tests/test_gpu_msm_prep.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_x4.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_x4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python3 tools/lib_ab.py 0g-ec-gpu_amd/lib_old/libecgpu.so 0g-ec-gpu_amd/lib/libecgpu.so
