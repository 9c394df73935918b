"""The fused sample + gather's f16 frame copy (acme_replay_sample_gather_frames) and the
DQN learner reading it (acme_transition_batch.obs_f16): the copy is f16(byte) of exactly
the gathered o_tm1 / o_t rows, and a learner step on it is bit-identical to the step that
converts the uint8 batch itself (the dataset -> DQNLearner path of the bench)."""

import ctypes

import numpy as np
import pytest
import torch

from tests.test_replay_gpu import _native

pytestmark = pytest.mark.gpu


def _f16_of(u8: np.ndarray) -> np.ndarray:
    return u8.astype(np.float16).view(np.uint16)


@pytest.mark.parametrize("prioritized", [True, False])
def test_sample_gather_frames_writes_exact_f16(prioritized):
    from acme_amd._lib import lib
    rng = np.random.default_rng(2)
    fields = [28224, 4, 4, 4, 28224]
    cap, n, B = 600, 700, 37
    data = [rng.integers(0, 256, (n, b), dtype=np.uint8) for b in fields]
    r = _native(cap, fields, prioritized)
    r.insert(data, rng.uniform(0.1, 2.0, n))
    L = lib()
    info = r.alloc_sample_info(B)
    outs = [torch.zeros(B, b, dtype=torch.uint8, device="cuda") for b in fields]
    ptrs = (ctypes.c_void_p * len(outs))(*[x.data_ptr() for x in outs])
    raw = [info[k].data_ptr() for k in ("slots", "keys", "probabilities", "table_size",
                                          "priorities")]
    fb = torch.full((2 * B, fields[0]), -1, dtype=torch.int16, device="cuda")
    assert L.acme_replay_sample_gather_frames(r.handle, B, 5, *raw, ptrs, fb.data_ptr(),
                                              None) == 0
    torch.cuda.synchronize()
    keys = info["keys"].cpu().numpy().view(np.int64)
    o_tm1, o_t = outs[0].cpu().numpy(), outs[4].cpu().numpy()
    np.testing.assert_array_equal(o_tm1, data[0][keys])
    np.testing.assert_array_equal(o_t, data[4][keys])
    got = fb.cpu().numpy().view(np.uint16)
    np.testing.assert_array_equal(got[:B], _f16_of(o_tm1))
    np.testing.assert_array_equal(got[B:], _f16_of(o_t))
    # Other layouts are refused.
    r2 = _native(cap, [64, 4], prioritized)
    r2.insert([rng.integers(0, 256, (10, 64), dtype=np.uint8),
               rng.integers(0, 256, (10, 4), dtype=np.uint8)], np.ones(10))
    outs2 = [torch.zeros(B, b, dtype=torch.uint8, device="cuda") for b in (64, 4)]
    ptrs2 = (ctypes.c_void_p * 2)(*[x.data_ptr() for x in outs2])
    info2 = r2.alloc_sample_info(B)
    raw2 = [info2[k].data_ptr() for k in ("slots", "keys", "probabilities", "table_size",
                                            "priorities")]
    assert L.acme_replay_sample_gather_frames(r2.handle, B, 5, *raw2, ptrs2, fb.data_ptr(),
                                              None) != 0


def test_learner_step_on_dataset_f16_frames_bitwise():
    from acme_amd.native import NativeDQN
    from acme_amd.networks import DQNAtariNetwork
    net = DQNAtariNetwork(18)
    B = 40
    rng = np.random.default_rng(9)
    a = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8")
    b = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8")
    p0, t0 = net.init(1), net.init(2)
    a.set_params(p0, t0)
    b.set_params(p0, t0)
    for _ in range(2):
        o1 = torch.from_numpy(rng.integers(0, 256, (B, 84 * 84 * 4), dtype=np.uint8)).cuda()
        o2 = torch.from_numpy(rng.integers(0, 256, (B, 84 * 84 * 4), dtype=np.uint8)).cuda()
        act = torch.from_numpy(rng.integers(0, 18, B).astype(np.int32)).cuda()
        rew = torch.from_numpy(rng.standard_normal(B).astype(np.float32)).cuda()
        dis = torch.full((B,), 0.99 ** 4, dtype=torch.float32, device="cuda")
        pr = torch.from_numpy(rng.uniform(1e-6, 1e-3, B)).cuda()
        fb = torch.cat([o1, o2]).to(torch.float16).view(torch.int16).contiguous()
        a.step(o1, act, rew, dis, o2, pr)
        b.step(o1, act, rew, dis, o2, pr, obs_f16=fb)
        torch.cuda.synchronize()
        assert a.loss.item() == b.loss.item()
        for buf in ("params", "m", "v", "grads"):
            ga, gb = a.get_params(buf), b.get_params(buf)
            for k in ga:
                np.testing.assert_array_equal(ga[k], gb[k], err_msg=f"{buf}/{k}")
