"""Achievable HBM bandwidth on this box ("also measure a
copy-kernel peak"): tools/native/hbm_peak.hip -- a dwordx4 streaming read
(partial sums) and a dwordx4 copy over 4 GiB, HIP events over 10 repetitions
-- beside torch's own copy_ and sum.  Build: hipcc --offload-arch=gfx950 -O3
-shared -fPIC -o tools/native/libhbm_peak.so tools/native/hbm_peak.hip"""
import ctypes
import json
import os
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
dev = torch.device("cuda", 0)
nbytes = 4 << 30
a = torch.ones(nbytes // 4, dtype=torch.float32, device=dev)
b = torch.empty_like(a)
lib = ctypes.CDLL(os.path.join(HERE, "native", "libhbm_peak.so"))
rd, cp = ctypes.c_float(), ctypes.c_float()
rc = lib.hbm_peak(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), ctypes.c_size_t(nbytes), 10,
                  ctypes.byref(rd), ctypes.byref(cp))
assert rc == 0


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


out = torch.empty((), dtype=torch.float32, device=dev)
res = {"hip_read_GBps": nbytes / (rd.value / 1e3) / 1e9, "hip_copy_GBps": 2 * nbytes / (cp.value / 1e3) / 1e9,
       "torch_copy_GBps": 2 * nbytes / timed(lambda: b.copy_(a)) / 1e9,
       "torch_sum_GBps": nbytes / timed(lambda: torch.sum(a, dim=0, out=out)) / 1e9,
       "bytes": nbytes}
print(json.dumps(res))
