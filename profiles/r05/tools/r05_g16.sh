# Round 5: the f32 engine's register ring (default) against the round-4 loop (r0): D4PG and
# IMPALA step time.
set -u
O=gpurun_out/r05g16; mkdir -p $O
W=d4pg VARS="r0" timeout -k 10 600 bash tools/ab_libs.sh $O/ab_d4pg > $O/ab_d4pg.log 2>&1; cat $O/ab_d4pg.log
W=impala VARS="r0" timeout -k 10 600 bash tools/ab_libs.sh $O/ab_impala > $O/ab_impala.log 2>&1; cat $O/ab_impala.log
