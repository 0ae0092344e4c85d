set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final2_smoke.log 2>&1 || { tail -20 gpurun_out/final2_smoke.log; exit 1; }
tail -2 gpurun_out/final2_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/final2_bench.log 2>&1 || { tail -20 gpurun_out/final2_bench.log; exit 1; }
grep '^{' gpurun_out/final2_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['roofline']['phases'].items()}, d['roofline']['frac'], d['cpu_baseline']['value'])"
