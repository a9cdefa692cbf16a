#!/bin/bash
# k_seg_apply at 1024 vs 512 threads per workgroup (libhstream_gpu_s512.so: -DHSG_SEG_NT=512):
# the C3 line with each library; the default library is put back afterwards.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof; export TMPDIR=/tmp
run() {
  timeout -k 10 300 python bench.py --config C3 --steps 4 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_seg_$1.log 2>&1 || { tail -20 gpurun_out/b_seg_$1.log; return 1; }
  tail -1 gpurun_out/b_seg_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3 $1', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
}
run nt1024 || exit 1
cp hstream_amd/libhstream_gpu.so /tmp/lib1024.so && cp hstream_amd/libhstream_gpu_s512.so hstream_amd/libhstream_gpu.so
run nt512; rc=$?
cp /tmp/lib1024.so hstream_amd/libhstream_gpu.so
[ $rc -eq 0 ] || exit $rc
run nt1024b
