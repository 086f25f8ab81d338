set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests/test_gpu_dist.py -x -q -m gpu > gpurun_out/pytest_dist.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_dist.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 tools/dist_rehearsal.py > gpurun_out/rehearsal1.log 2>&1; echo "rehearsal world1 rc=$?"; tail -3 gpurun_out/rehearsal1.log
timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-aux > gpurun_out/bench_torchrun1.log 2>&1; echo "bench torchrun1 rc=$?"; tail -1 gpurun_out/bench_torchrun1.log
timeout -k 10 180 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 tools/dist_rehearsal.py > gpurun_out/rehearsal2.log 2>&1; echo "rehearsal world2 (2 ranks, 1 GPU) rc=$?"; grep -E "rank|Error|error|Duplicate" gpurun_out/rehearsal2.log | head -12
exit 0
