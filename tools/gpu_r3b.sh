#!/bin/bash
# Round 3: the default bench line (C2 + configs), one-step kernel/copy timelines of C2 and C3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 550 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail gpurun_out/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench.json'))
print('C2', d.get('value'), d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('state_check'))
for k,v in (d.get('configs') or {}).items(): print(k, v['value'], v['ms_per_step'], v.get('checks'), v.get('wall_s'), (v.get('cpu_baseline') or {}).get('value'))
"
./tools/step_trace.sh > gpurun_out/steptrace.txt 2>&1 || { echo "step trace failed"; tail gpurun_out/steptrace.txt; exit 1; }
tail -45 gpurun_out/steptrace.txt
./tools/c3_trace.sh > gpurun_out/c3trace.txt 2>&1 || { echo "c3 trace failed"; tail gpurun_out/c3trace.txt; exit 1; }
echo c3 trace ok
