# A/B of trainer env knobs on the default bench (alternating, 2 rounds):
#   bash tools/ab_env.sh OUTDIR "A_ENV" "B_ENV" ...   (each arg: space-separated VAR=VAL list)
set -o pipefail
O=$1; shift
mkdir -p $O
for round in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --no-kernel-timing --steps 500 --warmup 50 > $O/ab_${i}_r${round}.json 2> $O/ab_${i}_r${round}.err || { echo "fail $cfg"; tail -5 $O/ab_${i}_r${round}.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/ab_${i}_r${round}.json').read().strip().splitlines()[-1]); print('r$round', '$cfg', d['value'], d['ms_per_step'], d['ms_per_step_p10_p50_p90'])"
  done
done
