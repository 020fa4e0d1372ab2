set -o pipefail
mkdir -p gpurun_out
for g in "" "--graph"; do
  timeout -k 10 300 python -u bench.py $g --no-cpu-baseline --no-score --no-c4 --no-dropin > gpurun_out/graph_bench$g.log 2>&1 || { tail -20 gpurun_out/graph_bench$g.log; exit 1; }
  grep '^{' gpurun_out/graph_bench$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$g', d['ms_per_step'], d['config']['launch'], d.get('c2_bf16_tables',{}).get('ms_per_step'))"
done
