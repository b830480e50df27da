# round 5: two-layer against one-layer bricks at r3 now that the one-layer
# kernels run 4 (FP64) / 5 (FP32) waves
set -o pipefail
mkdir -p gpurun_out/r5s
for rep in 1 2; do
  for tl in 0 1; do
    for pr in f32 f64; do
      GLS_TWO_LAYER=$tl timeout -k 10 150 python3 scripts/time_vmult.py input_hoffmann_3D_Re3900.json 3 $pr 30 | sed "s/^/two_layer=$tl /" || exit 1
      GLS_TWO_LAYER=$tl timeout -k 10 150 python3 scripts/time_vmult.py input_sphere_amg.json 3 $pr 20 | sed "s/^/two_layer=$tl /" || exit 1
    done
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5s/two_layer_r3.txt
