set -eo pipefail
mkdir -p gpurun_out/abp
for r in 1 2 3; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-check --steps 30 > gpurun_out/abp/prof_$r.json 2>/dev/null
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-check --steps 30 --no-prof > gpurun_out/abp/noprof_$r.json 2>/dev/null
done
for f in gpurun_out/abp/*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],3))"; done
