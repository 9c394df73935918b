# Round-6 call 2: MFMA rounding probes + accumulation variants; the B=64 gradient error structure.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g2; mkdir -p $O
timeout -k 10 120 tools/mfma_bias > $O/mfma_bias.log 2>&1 || { cat $O/mfma_bias.log; exit 3; }
cat $O/mfma_bias.log
timeout -k 10 300 python -u tools/grad_err_diag.py --B 64 --out $O > $O/graderr_B64.log 2>&1 || { tail -20 $O/graderr_B64.log; exit 4; }
grep -E "structure|wgrad|plane:|f32:|conv2_d" $O/graderr_B64.log
