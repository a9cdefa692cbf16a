cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1
bash tools/pmc.sh c2agg "k_part_agg" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" -- --config C2
timeout -k 10 300 python bench.py --config C2 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_c2.log 2>&1; cut -c1-300 gpurun_out/bench_c2.log
timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_c5.log 2>&1; cut -c1-300 gpurun_out/bench_c5.log
