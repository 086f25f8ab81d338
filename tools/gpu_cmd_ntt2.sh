set -o pipefail
timeout -k 10 900 python3 tools/lib_ab.py 0g-ec-gpu_amd/lib_old/libecgpu.so 0g-ec-gpu_amd/lib/libecgpu.so
