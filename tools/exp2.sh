cd /root/repo; export TMPDIR=/tmp
for v in "" "HSG_NOPACK=1"; do env $v HSG_PHASES=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/exp2.log 2>&1 || exit 1; echo "== $v"; grep "agg wg\|scatter wg" gpurun_out/exp2.log | tail -2; grep '^{' gpurun_out/exp2.log | cut -c1-100; done
