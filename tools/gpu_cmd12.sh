set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python3 tools/lib_ab.py 0g-ec-gpu_amd/lib/libecgpu.so 0g-ec-gpu_amd/lib_w3/libecgpu.so 0g-ec-gpu_amd/lib_w4/libecgpu.so > gpurun_out/lib_ab.log 2>&1; echo "lib_ab rc=$?"; cat gpurun_out/lib_ab.log
