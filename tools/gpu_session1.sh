cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -k "not c4_full" -x -v --timeout 300 --timeout-method thread > gpurun_out/t_configs.log 2>&1; echo "configs rc=$?"; tail -12 gpurun_out/t_configs.log
bash tools/prof.sh c3 --config C3 --records 100000000 && bash tools/prof.sh c4 --config C4 --records 33554432 && bash tools/prof.sh c5 --config C5
