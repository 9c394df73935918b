"""Phase stamps of the online fc_fwd, conv1_fwd, conv2_fwd and conv3_fwd launches (gemm_p3.h HasStamps; ACME_V_STAMPS=1): the
bench's DQN learner runs a few steps, then each workgroup's entry / exit (s_memrealtime,
100 MHz, comparable across workgroups) and its prologue, k loop and epilogue lengths
(s_memtime, shader clocks) are summarised.  Run under gpurun: python3 tools/gemm_stamps.py"""
import os
import sys

import numpy as np

os.environ["ACME_V_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from acme_amd.native import NativeDQN
    from acme_amd.networks import DQNAtariNetwork
    B = 512
    net = DQNAtariNetwork(18)
    d = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8")
    d.set_params(net.init(1), net.init(2))
    g = torch.Generator(device="cuda").manual_seed(0)
    o = torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device="cuda", generator=g)
    o2 = torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device="cuda", generator=g)
    a = torch.randint(0, 18, (B,), dtype=torch.int32, device="cuda", generator=g)
    r = torch.randn(B, device="cuda", generator=g)
    dd = torch.full((B,), 0.99, device="cuda")
    pr = torch.full((B,), 1e-4, dtype=torch.float64, device="cuda")
    for _ in range(5):
        d.step(o, a, r, dd, o2, pr)
    torch.cuda.synchronize()
    allst = d.debug_buffer("gemm_stamps").view(np.int64).reshape(4, 4096, 8)
    for name, st in zip(("fc_fwd (online)", "conv1_fwd", "conv2_fwd", "conv3_fwd (online)"),
                        allst):
        st = st[st[:, 0] != 0]
        if not len(st):
            continue
        rt0, rt1, t0, t1, t2, t3 = (st[:, i].astype(np.float64) for i in range(6))
        mhz = np.median((t3 - t0) / ((rt1 - rt0) * 10e-3))  # shader clocks per us
        print(f"{name}: {len(st)} workgroups; shader clock {mhz:.0f} MHz (median); launch "
              f"span {(rt1.max() - rt0.min()) * 0.01:.1f} us, entry spread "
              f"{(rt0.max() - rt0.min()) * 0.01:.1f} us, exit spread "
              f"{(rt1.max() - rt1.min()) * 0.01:.1f} us")
        for ph, v in (("prologue (to first barrier)", t1 - t0), ("k loop", t2 - t1),
                      ("epilogue", t3 - t2), ("total", t3 - t0)):
            us = v / mhz
            print(f"  {ph:28s} median {np.median(us):6.2f} us  min {us.min():6.2f}  max "
                  f"{us.max():6.2f}")

if __name__ == "__main__":
    main()
