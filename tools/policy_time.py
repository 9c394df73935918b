"""Times IMPALA's batched policy step (acme_impala_policy_step, the actors' network call)
alone on the GPU: wall time per call through IMPALALearner.pipelined_policy at `rows` rows,
and the library's section profile of one call.  Usage: python tools/policy_time.py [rows]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from acme_amd import _lib, specs  # noqa: E402
from acme_amd.agents.impala import IMPALALearner  # noqa: E402
from acme_amd.networks import IMPALAAtariNetwork  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 32
net = IMPALAAtariNetwork(18)
spec = specs.EnvironmentSpec(observations=None, actions=None, rewards=None, discounts=None)
learner = IMPALALearner(spec, net, iter(()), learning_rate=1e-3, batch_size=16,
                        sequence_length=20)
pol = learner.pipelined_policy(rows)
rng = np.random.default_rng(0)
obs = rng.integers(0, 256, (rows, 84, 84, 4), dtype=np.uint8)
pa = np.zeros(rows, np.int32)
pr = np.zeros(rows, np.float32)
h = np.zeros((rows, 256), np.float32)
for _ in range(20):
    pol.issue(obs, pa, pr, h, h)
    pol.result()
t0 = time.perf_counter()
n = 200
for _ in range(n):
    pol.issue(obs, pa, pr, h, h)
    pol.result()
print(f"rows {rows}: {1e6 * (time.perf_counter() - t0) / n:.1f} us per issue+result")
_lib.set_profiling(True)
_lib.lib().acme_profile_reset()
for _ in range(10):
    pol.issue(obs, pa, pr, h, h)
    pol.result()
torch.cuda.synchronize()
_lib.set_profiling(False)
import ctypes  # noqa: E402
L = _lib.lib()
for i in range(L.acme_profile_num_sections()):
    nm, ms, cnt = ctypes.c_char_p(), ctypes.c_double(), ctypes.c_int64()
    fl, by = ctypes.c_double(), ctypes.c_double()
    L.acme_profile_query(i, ctypes.byref(nm), ctypes.byref(ms), ctypes.byref(cnt),
                         ctypes.byref(fl), ctypes.byref(by))
    if cnt.value:
        print(f"{nm.value.decode():28s} {1e3 * ms.value / cnt.value:8.2f} us")
