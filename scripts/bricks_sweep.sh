cd $GRAFT_REPO_ROOT
for b in 4,4,2 4,4,1 4,2,1 2,1,1; do
  timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --brick $b > gpurun_out/br_$b.json 2>gpurun_out/br_$b.err || exit 1
  echo "$b $(python -c "import json;d=json.load(open('gpurun_out/br_$b.json'));print(d['ms_per_step']*1e3)")"
done
