# round-6 GPU batch f: accumulation segments fitted to whole rounds (new lib) vs the previous build
set -o pipefail
mkdir -p gpurun_out
B=$PWD/0g-ec-gpu_amd/lib_ab/libecgpu_base.so
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_msm.py tests/test_gpu_dist.py -x -q --timeout 300 -k "2p20 or kat or skew or cycled or grid or config4 or dist" > gpurun_out/pytest_fitseg.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_fitseg.log; [ $rc -eq 0 ] || exit $rc
for C in bls12_381 bn254; do
  ECGPU_LIB=$B timeout -k 10 300 python3 -u tools/grid_split_probe.py 26 $C 3 > gpurun_out/fitseg_probe_base_$C.log 2>&1 || exit 1
  timeout -k 10 300 python3 -u tools/grid_split_probe.py 26 $C 3 > gpurun_out/fitseg_probe_new_$C.log 2>&1 || exit 1
  tail -3 gpurun_out/fitseg_probe_base_$C.log | cut -c1-400; tail -3 gpurun_out/fitseg_probe_new_$C.log | cut -c1-400
done
for L in 20 26; do
  timeout -k 10 400 python3 -u tools/msm_ab.py $L "" "ECGPU_LIB=$B" > gpurun_out/fitseg_ab_bls_$L.log 2>&1 || exit 1; cat gpurun_out/fitseg_ab_bls_$L.log
  AB_CURVE=bn254 timeout -k 10 400 python3 -u tools/msm_ab.py $L "" "ECGPU_LIB=$B" > gpurun_out/fitseg_ab_bn_$L.log 2>&1 || exit 1; cat gpurun_out/fitseg_ab_bn_$L.log
done
