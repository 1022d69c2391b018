#!/bin/bash
# Same-box A/B of the host-buffer upload (bench.py host_buffers leg): chunk sizes / host threads
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in ${AB:-"CE_UPLOAD_CHUNK=67108864"}; do
  echo -n "$v "
  env ${v//,/ } timeout -k 10 300 python bench.py --configs '' --no-cpu --no-variant-b --steps 3 --warmup 1 > gpurun_out/up.json 2> gpurun_out/up.err || { echo failed; tail -3 gpurun_out/up.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/up.json'))['host_buffers'];print(d['value'], d['pcie_GBps'], d['upload_ms'], d['ms_per_step'])"
done
