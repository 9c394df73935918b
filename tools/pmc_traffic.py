#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE collected
in SEPARATE passes with --kernel-trace only, MI355X_MICROARCH.md § HBM):

  bytes_read  = 2 x FETCH_SIZE x 1024   (FETCH_SIZE is in KB and, on gfx950, reports half
                                        the bytes of wide 16-B-per-lane reads)
  bytes_write = WRITE_SIZE x 1024       (exact for 16-B-per-lane stores and float atomics;
                                        narrower stores are uncalibrated)

averaged per launch and keyed by the library's profiler section names (the names bench.py
reports), so bench.py can put the dominant kernel's measured traffic next to its
algorithmic bytes.  Usage:
    tools/pmc_traffic.py <workload> <fetch_dir> <write_dir> <out.json>
"""
import collections
import csv
import glob
import os
import json
import re
import sys

# kernel symbol pattern -> profiler section name (first match wins), per workload
# (Patterns see "<kernel name> grid=<Grid_Size>": the critic head and the policy's hidden
# layers are one instantiation of the direct engine, told apart by their grids.)
SECTIONS_D4PG = [
    (r"gemm_direct_kernel<16, 8, .*DenseFwd<.* grid=32768$", "d4pg_critic_head"),
    (r"gemm_direct_kernel<.*DenseFwd<true", "d4pg_mlp_fwd"),
    (r"gemm_direct_multi_kernel<\d+, 8, acme::gemm::ZSet<acme::conv::DenseDgrad<true>, 3>, "
     r"acme::gemm::ZSet<acme::conv::DenseWgrad<true, acme::conv::InF32>, 3> >", "d4pg_bwd_mlp"),
    (r"gemm_direct_multi_kernel<", "d4pg_bwd_heads_first"),
    # the staged engine (rounds 1-4, -DD4_DIRECT=0)
    (r"gemm_f32_kernel<32, 32, 1, 1, 16, 8, acme::gemm::ZSet<acme::conv::DenseFwd<true", "d4pg_mlp_fwd"),
    (r"gemm_f32_kernel<32, 32, 1, 1, 16, 8, acme::gemm::ZSet<acme::conv::DenseFwd<false", "d4pg_critic_head"),
    (r"gemm_f32_multi_kernel<.*ZSet<acme::conv::DenseDgrad<true", "d4pg_bwd_mlp"),
    (r"gemm_f32_multi_kernel<", "d4pg_bwd_heads_first"),
    (r"ln_bwd_kernel", "d4pg_ln_bwd"),
    (r"ln_first_kernel", "d4pg_ln_first"),
    (r"d4pg_loss_kernel", "d4pg_loss"),
    (r"grad_sumsq_kernel|clip_adam_kernel", "d4pg_adam"),
    (r"sample_gather_small_kernel", "replay_sample_gather"),
]
SECTIONS_IMPALA = [
    (r"P3DenseFwd", "impala_oar_fwd"),
    (r"P3DenseWgrad", "impala_wi_wgrad"),
    (r"P3DenseDgrad", "impala_feat_dgrad"),
    (r"oar_finish_kernel", "impala_oar_reduce"),
    (r"DenseDgrad<true", "impala_feat_dgrad"),
    (r"OarFwd", "impala_oar_fwd"),
    (r"OarWgrad", "impala_wi_wgrad"),
    (r"lstm_fwd_rg_kernel|lstm_fwd_step", "impala_lstm_fwd"),
    (r"lstm_bwd_rg_kernel|lstm_bwd_step", "impala_lstm_bwd"),
    (r"grad_sumsq_kernel|clip_adam_kernel", "impala_adam"),
    (r"ConvFwd<acme::conv::Geom<84,", "conv1_fwd"),
    (r"ConvFwd<acme::conv::Geom<21,", "conv2_fwd"),
    (r"ConvFwd<acme::conv::Geom<11,", "conv3_fwd"),
    (r"ConvWgrad<acme::conv::Geom<84,", "conv1_wgrad"),
    (r"ConvWgrad<acme::conv::Geom<21,", "conv2_wgrad"),
    (r"ConvWgrad<acme::conv::Geom<11,", "conv3_wgrad"),
    (r"ConvDgradSub", "conv2_dgrad"),
    (r"ConvDgrad<", "conv3_dgrad"),
]
SECTIONS = [
    (r"P3DenseFwd", "fc_fwd"),
    (r"P3DenseWgrad", "fc_wgrad"),
    (r"P3DenseDgrad", "fc_dgrad"),
    (r"fc_head_forward_kernel|fc_head1024_kernel", "fc_head_fwd"),
    (r"frames_f16_kernel", "frames_f16"),
    (r"head_dz_planes_kernel", "head_dz"),
    (r"dqn_loss_head_dz_kernel", "loss_head_dz"),
    (r"dqn_head_loss_dz_kernel", "head_loss_dz"),
    (r"gemm_p3c12_kernel", "conv12_fwd"),
    (r"gemm_\w+_kernel<128, 128, 2, 2,.*DenseFwd<true", "fc_fwd"),
    (r"ConvFwd<acme::conv::Geom<84,", "conv1_fwd"),
    (r"ConvFwd<acme::conv::Geom<21,", "conv2_fwd"),
    (r"ConvFwd<acme::conv::Geom<11,", "conv3_fwd"),
    (r"DenseWgrad<true", "fc_wgrad"),
    (r"DenseDgrad<true", "fc_dgrad"),
    (r"ConvWgrad<acme::conv::Geom<84,", "conv1_wgrad"),
    (r"ConvWgrad<acme::conv::Geom<21,", "conv2_wgrad"),
    (r"ConvWgrad<acme::conv::Geom<11,", "conv3_wgrad"),
    (r"ConvDgradSub", "conv2_dgrad"),
    (r"ConvDgrad<", "conv3_dgrad"),
    (r"(?<!clip_)adam_kernel|adam_slabs_kernel", "adam"),
    (r"sample_gather_pair_kernel|sample_gather_pipe_kernel", "replay_sample_gather"),
    (r"gather_fields_kernel|gather_pair_kernel|gather_pieces_kernel", "replay_gather"),
    (r"sample_prioritized_kernel", "replay_sample"),
    (r"prio_update_fused_kernel", "replay_update"),
]
SECTIONS_R2D2 = [
    # The Atari plane path (the bench's), then the f32 engine's names.
    (r"P3DenseFwd", "r2d2_oar_fwd"),
    (r"P3DenseWgrad", "r2d2_wi_wgrad"),
    (r"P3DenseDgrad", "r2d2_feat_dgrad"),
    (r"oar_finish_kernel", "r2d2_oar_reduce"),
    (r"oar_wgrad_tail_kernel", "r2d2_wi_wgrad_tail"),
    (r"r2d2_frames_f16_kernel", "r2d2_permute"),
    (r"split_planes_lagged_kernel", "r2d2_planes"),
    (r"DenseWgradRC", "r2d2_hidden_wgrad"),
    (r"lstm_fwd_rg_kernel", "r2d2_lstm_fwd"),
    (r"lstm_bwd_rg_kernel", "r2d2_lstm_bwd"),
    (r"OarFwd", "r2d2_oar_fwd"),
    (r"OarWgrad", "r2d2_wi_wgrad"),
    (r"HPrevTM", "r2d2_wh_wgrad"),
    (r"<64, 128, 2, 2,.*DenseDgrad<true", "r2d2_feat_dgrad"),
    (r"DenseDgrad<true", "r2d2_hidden_dgrad"),
    (r"DenseWgrad<true", "r2d2_hidden_wgrad"),
    (r"DenseFwd<true", "r2d2_hidden_fwd"),
    (r"DuelHeadFwd", "r2d2_head_fwd"),
    (r"DuelHeadWgrad", "r2d2_head_wgrad"),
    (r"lstm_fwd_step", "r2d2_lstm_fwd"),
    (r"lstm_bwd_step", "r2d2_lstm_bwd"),
    (r"r2d2_loss_kernel", "r2d2_loss"),
    (r"r2d2_permute_kernel", "r2d2_permute"),
    (r"(?<!clip_)adam_kernel", "r2d2_adam"),
] + [e for e in SECTIONS_IMPALA if e[1].startswith("conv")]
TABLES = {"dqn": SECTIONS, "d4pg": SECTIONS_D4PG, "impala": SECTIONS_IMPALA,
          "r2d2": SECTIONS_R2D2}
TABLE = SECTIONS


def section(name, grid=None):
    key = f"{name} grid={grid}" if grid is not None else name
    for pat, sec in TABLE:
        if re.search(pat, key):
            return sec
    return None


def per_launch(d, counter):
    # The newest pass only: gpurun merges each run's output into the same local directory.
    paths = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    paths = sorted(paths, key=os.path.getmtime)[-1:]
    vals = collections.defaultdict(list)
    for path in paths:
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != counter:
                continue
            sec = section(r["Kernel_Name"], r.get("Grid_Size"))
            if sec:
                vals[sec].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    global TABLE
    workload, fetch_dir, write_dir, out = sys.argv[1:5]
    TABLE = TABLES[workload]
    f = per_launch(fetch_dir, "FETCH_SIZE")
    w = per_launch(write_dir, "WRITE_SIZE")
    res = {}
    for sec in sorted(set(f) | set(w)):
        rd = 2.0 * 1024.0 * f.get(sec, 0.0)
        wr = 1024.0 * w.get(sec, 0.0)
        res[sec] = {"read_bytes": round(rd), "write_bytes": round(wr), "bytes": round(rd + wr)}
    json.dump({"method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; "
                         "read = 2 x FETCH_SIZE KB (gfx950 half-count of 16-B reads), write = "
                         "WRITE_SIZE KB; per launch", "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:22s} {v['bytes'] / 1e6:10.1f} MB/launch")


if __name__ == "__main__":
    main()
