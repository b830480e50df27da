# round 5: brick shape A/B at r2 (4x4x1 layers vs 4x2x1 half layers), FP32 and FP64
set -o pipefail
mkdir -p gpurun_out/r5o
for rep in 1 2; do
  for sh in 4,4,1 4,2,1; do
    for pr in f32 f64; do
      timeout -k 10 120 python3 scripts/time_vmult.py input_hoffmann_3D_Re3900.json 2 $pr 100 $sh || exit 1
    done
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5o/brick_shape_ab.txt
