# round 5: two-layer (4x4x2) bricks at r2 against one-layer layers, FP32 and FP64
set -o pipefail
mkdir -p gpurun_out/r5p
for rep in 1 2; do
  for tl in 0 1; do
    for pr in f32 f64; do
      GLS_TWO_LAYER=$tl timeout -k 10 120 python3 scripts/time_vmult.py input_hoffmann_3D_Re3900.json 2 $pr 100 | sed "s/^/two_layer=$tl /" || exit 1
    done
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5p/two_layer_r2.txt
