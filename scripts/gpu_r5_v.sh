# round 5 prototype: 512-thread (8-wave) workgroups, two-layer 4x4x2 bricks
# in 2 rounds (lib/var/blk512.so, BLOCK = 512 build) against the default
set -o pipefail
mkdir -p gpurun_out/r5v
V=dealii-ns-gls_amd/lib/var/blk512.so
run() { # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-companions > gpurun_out/r5v/$label.json 2> gpurun_out/r5v/$label.err || { echo "$label failed"; tail -5 gpurun_out/r5v/$label.err; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r5v/$label.json'));print('$label', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('parity',{}), d['config'].get('brick_shape'))"
}
for rep in 1 2; do
  run default_$rep GLS_X=0 || exit 1
  run blk512_one_$rep GLS_AMD_LIB=$V GLS_TWO_LAYER=0 || exit 1
  run blk512_two_$rep GLS_AMD_LIB=$V GLS_TWO_LAYER=1 || exit 1
done 2>&1 | tee gpurun_out/r5v/summary.txt
for tl in 0 1; do GLS_AMD_LIB=$V GLS_TWO_LAYER=$tl timeout -k 10 120 python3 scripts/time_vmult.py input_hoffmann_3D_Re3900.json 2 f32 100 | sed "s/^/blk512 two_layer=$tl /"; done 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r5v/summary.txt
