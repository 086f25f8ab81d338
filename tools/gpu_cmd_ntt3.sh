set -o pipefail
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fft.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ntt.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_ntt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 tools/ntt_ab.py ECGPU_LIB=0g-ec-gpu_amd/lib_lb/libecgpu.so ECGPU_LIB=0g-ec-gpu_amd/lib/libecgpu.so ECGPU_LIB=0g-ec-gpu_amd/lib/libecgpu.so,ECG_NTT_TILE=11
