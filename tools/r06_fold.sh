#!/bin/bash
# round 6: the C3 fold's aligned reservations -- fold tests, kernel-stat A/B (align off/on),
# FETCH/WRITE traffic of both
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dotset.py -k "partitioned or adds_without_sort or local_apply or kway" > gpurun_out/fold_tests.log 2>&1 || { tail -30 gpurun_out/fold_tests.log; exit 1; }
tail -1 gpurun_out/fold_tests.log
for A in 0 1; do
  bash tools/c3_kstats.sh align$A CE_DS_PART_ALIGN=$A | grep -E "total|part_|kput|khold|kfinal|contig" || exit 1
done
for A in 0 1; do
  CE_DS_PART_ALIGN=$A bash tools/c3_traffic.sh > gpurun_out/c3traffic_align$A.txt || exit 1
  cp gpurun_out/c3traffic/c3_traffic.json gpurun_out/c3_traffic_align$A.json
  python3 -c "
import json;d=json.load(open('gpurun_out/c3_traffic_align$A.json'))['kernels']
f=['k_ds_contig','k_ds_part_adds','k_ds_part_kills','k_ds_part_apply','k_ds_clock']
t=0
for k in f:
  x=d.get(k,{});a=x.get('fetch_size_bytes',0)/1e6;b=x.get('write_size_bytes',0)/1e6;t+=a+b;print('$A',k,round(a,1),round(b,1))
print('$A fold total MB',round(t,1))
for k in ['k_ds_kput','k_ds_khold','k_ds_kfinal']:
  x=d.get(k,{});print('$A',k,round(x.get('fetch_size_bytes',0)/1e6,1),round(x.get('write_size_bytes',0)/1e6,1))
"
done
