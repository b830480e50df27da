# round 5: cost of the deterministic mode (GLS_DETERMINISTIC), r2 FP64 / FP32 vmult
set -o pipefail
mkdir -p gpurun_out/r5aa
for rep in 1 2; do
  for pr in f64 f32; do
    timeout -k 10 120 python3 scripts/time_vmult.py input_hoffmann_3D_Re3900.json 2 $pr 100 - | sed 's/^/default /' || exit 1
    timeout -k 10 120 python3 scripts/time_vmult.py input_hoffmann_3D_Re3900.json 2 $pr 100 - det | sed 's/^/deterministic /' || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5aa/det_cost.txt
