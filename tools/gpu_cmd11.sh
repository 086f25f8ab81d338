set -o pipefail
mkdir -p gpurun_out
ECGPU_LIB=$PWD/0g-ec-gpu_amd/lib_nv/libecgpu.so timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > gpurun_out/pytest_nv.log 2>&1; rc=$?; echo "pytest(nv) rc=$rc"; tail -3 gpurun_out/pytest_nv.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 tools/lib_ab.py 0g-ec-gpu_amd/lib/libecgpu.so 0g-ec-gpu_amd/lib_nv/libecgpu.so > gpurun_out/lib_ab.log 2>&1; echo "lib_ab rc=$?"; cat gpurun_out/lib_ab.log
