set -e
# A/B of the select-ahead split: parts merged by k_fixlist<PARTS> before its wait (1) or by the select's last part (0)
mkdir -p gpurun_out/ab
for rep in 1 2; do
for v in 1 0; do
  KOORDEVAL_FIX_MERGE=$v timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --stream-nodes 0 > gpurun_out/ab/m${v}_r${rep}.json 2> gpurun_out/ab/m${v}_r${rep}.err
  python -c "import json;d=json.load(open('gpurun_out/ab/m${v}_r${rep}.json'));print('fix_merge',${v},'rep',${rep},round(d['value']/1e9,2),'G eval',round(d['kernel_ms']['eval']*1e3,1),'sel',round(d['kernel_ms']['select']*1e3,1),'handoff',round(d['kernel_ms']['handoff']*1e3,1),'resolve',round(d['kernel_ms']['resolve']*1e3,1),'parity',d.get('parity'))"
done; done
