"""Multi-rank rehearsal of the native RCCL path on whatever GPUs are visible
(dev tool).  Launch: torchrun --nproc-per-node N --master-addr 127.0.0.1
tools/dist_rehearsal.py.  Ranks map to device LOCAL_RANK % device_count, so on a
single-GPU box all ranks share GPU 0 (RCCL may refuse that: the point is to
find out).  Checks ecg_msm_dist and ecg_fft_dist against single-GPU results."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "0g-ec-gpu_amd")]
import ecgpu  # noqa: E402
from ecgpu import dist as edist  # noqa: E402

group = edist.HostGroup.from_env()
rank, world = group.rank, group.world
ndev = ecgpu.lib().ecg_device_count()
prog = ecgpu.program(ecgpu.Device(int(os.environ.get("LOCAL_RANK", "0")) % ndev))
print(f"rank {rank}: {ecgpu.lib().ecg_runtime_info().decode()}", flush=True)
edist.comm_init(prog, rank, world, group.broadcast)
print(f"rank {rank}/{world}: comm up on device {prog.device.index}", flush=True)
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
log_n = 16
n = 1 << log_n
m = n // world
rng = np.random.default_rng(9)
a = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
a[:, 3] &= np.uint64(2**62 - 1)
w = pow(7, (R - 1) >> 32, R)
for _ in range(log_n, 32):
    w = w * w % R
om = np.array([((w << 256) % R >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)
d = ecgpu.DeviceBuffer.upload(prog, np.ascontiguousarray(a[rank * m:(rank + 1) * m]))
edist.fft_dist(prog, "bls12_381_fr", d, om, log_n)
full = a.copy()
dref = ecgpu.DeviceBuffer.upload(prog, full)
ecgpu.fft_dev(prog, "bls12_381_fr", dref, om, log_n)
ok_fft = bool((d.read(shape=(m, 4)) == dref.read(shape=(n, 4))[rank * m:(rank + 1) * m]).all())
nm = 1 << 16
per = nm // world
bases = ecgpu.gen_bases_dev(prog, "bls12_381", 5 + rank * per * 3, 3, per)
e = rng.integers(0, 2**64, size=(nm, 4), dtype=np.uint64)
e[:, 3] &= np.uint64(2**62 - 1)
d_e = ecgpu.DeviceBuffer.upload(prog, np.ascontiguousarray(e[rank * per:(rank + 1) * per]))
got = edist.msm_dist(prog, "bls12_381", bases, d_e, per)
all_b = ecgpu.gen_bases_dev(prog, "bls12_381", 5, 3, nm)
d_all = ecgpu.DeviceBuffer.upload(prog, e)
want = ecgpu.msm_dev(prog, "bls12_381", all_b, d_all, nm)
ok_msm = bool((got == want).all())
print(f"rank {rank}: fft_dist ok={ok_fft} msm_dist ok={ok_msm}", flush=True)
group.barrier()
ecgpu.lib().ecg_comm_destroy(prog.handle)
group.close()
sys.exit(0 if (ok_fft and ok_msm) else 1)
