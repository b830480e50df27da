# round 5: the revised two-layer rule -- Re3900 r3, sphere r3, Turek-3D r3
# by default (which layout each takes), and the Turek-3D V-cycle
set -o pipefail
mkdir -p gpurun_out/r5t
for rep in 1 2; do
  for deck in input_hoffmann_3D_Re3900.json input_sphere_amg.json input_turek_3D_Re100.json; do
    for pr in f32 f64; do
      timeout -k 10 150 python3 scripts/time_vmult.py $deck 3 $pr 20 || exit 1
    done
  done
  GLS_TWO_LAYER=1 timeout -k 10 150 python3 scripts/time_vmult.py input_turek_3D_Re100.json 3 f32 20 | sed 's/^/forced two-layer: /' || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5t/two_layer_rule.txt
