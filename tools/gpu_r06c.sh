# round-6 GPU batch c: accumulate with entries two ahead (new lib) vs the previous build, both curves
set -o pipefail
mkdir -p gpurun_out
B=$PWD/0g-ec-gpu_amd/lib_ab/libecgpu_base.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_msm.py -x -q --timeout 200 -k "2p20 or kat or skew or cycled" > gpurun_out/pytest_msm_c.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_msm_c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/msm_ab.py 26 "" "ECGPU_LIB=$B" > gpurun_out/prefetch2_ab_bls.log 2>&1; rc=$?; cat gpurun_out/prefetch2_ab_bls.log; [ $rc -eq 0 ] || exit $rc
AB_CURVE=bn254 timeout -k 10 400 python3 -u tools/msm_ab.py 26 "" "ECGPU_LIB=$B" > gpurun_out/prefetch2_ab_bn.log 2>&1; rc=$?; cat gpurun_out/prefetch2_ab_bn.log
