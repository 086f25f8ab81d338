# round-6 GPU batch b: BN254 accumulate at 2 waves/SIMD (A/B) + self-launched N=4 rehearsal
set -o pipefail
mkdir -p gpurun_out
AB_CURVE=bn254 timeout -k 10 400 python3 -u tools/msm_ab.py 26 "" "ECGPU_LIB=$PWD/0g-ec-gpu_amd/lib_ab/libecgpu_accw2.so" > gpurun_out/bn254_accw2_ab.log 2>&1; rc=$?
cat gpurun_out/bn254_accw2_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --gpus 4 --transport host --single-device --steps 3 --warmup 1 --ntt-log 20 --no-cpu-baseline > gpurun_out/rehearsal_4_selflaunch.log 2>&1; echo rehearsal rc=$?
tail -c 600 gpurun_out/rehearsal_4_selflaunch.log
