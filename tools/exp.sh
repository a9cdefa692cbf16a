cd /root/repo; export TMPDIR=/tmp
for x in ${EXPS:-0 1 2}; do HSG_EXP=$x HSG_PHASES=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/exp_$x.log 2>&1 || exit 1; echo "== exp $x"; grep "agg wg" gpurun_out/exp_$x.log | tail -1; grep '^{' gpurun_out/exp_$x.log | cut -c1-120; done
