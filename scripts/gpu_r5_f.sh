# round 5: one-layer 4-wave vs two-layer 3-wave FP64 bricks on the r3 meshes
set -o pipefail
for rep in 1 2; do
  for tl in default 0; do
    for spec in "input_hoffmann_3D_Re3900.json 3 f64" "input_sphere_amg.json 3 f64" "input_hoffmann_3D_Re3900.json 3 f32"; do
      if [ $tl = default ]; then E=""; else E="GLS_TWO_LAYER=0"; fi
      echo -n "two_layer=$tl "; env $E timeout -k 10 120 python scripts/time_vmult.py $spec 50 || exit 1
    done
  done
done
