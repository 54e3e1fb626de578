set -e
out=gpurun_out/prio.jsonl
: > $out
for r in 1 2; do
for P in none tb_low dp_high both; do
  SED_STREAM_PRIO=$P timeout -k 10 200 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline > gpurun_out/p.json 2> gpurun_out/p.log
  python3 -c "import json; d=json.load(open('gpurun_out/p.json')); print(json.dumps({'prio':'$P','value':d['value'],'ms_step':d['ms_per_step'],'dp_ms':d['roofline']['kernel_ms'],'tb_ms':d['traceback_ms']}))" >> $out
done
done
