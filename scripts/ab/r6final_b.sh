# round 6 final evidence, part B: the default bench line, rocprofv3 stats of the bench command, PMC of the FP64 and FP32 r2 kernels
bash scripts/gpu_run.sh r6final bench stats pmc:f64 pmc:f32
