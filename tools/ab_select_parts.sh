set -e
mkdir -p gpurun_out/ab
for rep in 1 2; do
for p in 4 1 2; do
  KOORDEVAL_SELECT_PARTS=$p timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --stream-nodes 0 > gpurun_out/ab/p${p}_r${rep}.json 2> gpurun_out/ab/p${p}_r${rep}.err
  python -c "import json,sys;d=json.load(open('gpurun_out/ab/p${p}_r${rep}.json'));k=d['roofline'].get('kernels',{});print('parts',${p},'rep',${rep},round(d['value']/1e9,2),'G eval',round(d['kernel_ms']['eval']*1e3,1),'sel',round(d['kernel_ms']['select']*1e3,1),'handoff',round(d['kernel_ms']['handoff']*1e3,1),'resolve',round(d['kernel_ms']['resolve']*1e3,1))"
done; done
