# BN254 / BLS12-381 accumulate at a 4-wave register cap (A/B build lib_ab/libecgpu_w4.so)
set -o pipefail
R=$GRAFT_REPO_ROOT
W4=$R/0g-ec-gpu_amd/lib_ab/libecgpu_w4.so
AB_CURVE=bn254 timeout -k 10 400 python3 tools/msm_ab.py 24 "" "ECGPU_LIB=$W4" > $R/gpurun_out/w4_bn24.log 2>&1; cat $R/gpurun_out/w4_bn24.log
timeout -k 10 400 python3 tools/msm_ab.py 24 "" "ECGPU_LIB=$W4" > $R/gpurun_out/w4_bls24.log 2>&1; cat $R/gpurun_out/w4_bls24.log
