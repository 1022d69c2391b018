#!/bin/bash
# Host-buffer path A/B (upload threads / chunk size): pcie GB/s and files/s per setting, twice.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for v in ${AB:-"CE_UPLOAD_THREADS=16 CE_UPLOAD_THREADS=12 CE_UPLOAD_THREADS=8"}; do
    echo -n "$v "
    env ${v//,/ } timeout -k 10 300 python bench.py --configs '' --no-cpu --no-variant-b --no-clock --steps 2 > gpurun_out/hb.json 2> gpurun_out/hb.err || { echo failed; tail -3 gpurun_out/hb.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/hb.json').read().strip().splitlines()[-1]);h=d['host_buffers'];print(h['pcie_GBps'], h['value'])"
  done
done
