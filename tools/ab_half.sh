set -o pipefail
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-pmc --mcmc-iters 0 --no-extra-configs --steps 20 --warmup 5"
for r in 1 2 3; do
  for f in "" "--half-waves"; do
    for w in 65536 131072; do
      timeout -k 10 90 $B --walkers $w $f > gpurun_out/ab_half_tmp.log 2>&1 || exit 1
      python -c "import json,sys;l=[x for x in open('gpurun_out/ab_half_tmp.log') if x.startswith('{')][-1];d=json.loads(l);print(json.dumps({'rep':$r,'flag':'$f','W':$w,'kernel_ms':d['roofline']['kernel_ms'],'frac':d['roofline']['frac'],'value':d['value']}))" >> gpurun_out/r02zp_ab_half.log
    done
  done
done
