"""The brick kernels' float quotient (csrc/brick.h idiv_f): floor(i / d) as
(int)(((float)i + 0.5f) * r) with r = 1.0f / (float)d computed on the host
(gls_op.hip brick_args), exact for every lattice index 0 <= i < 4096 and
every divisor 1 <= d <= 729 (lattice rows / planes, brick extents).
IEEE binary32 emulated with numpy float32 (the device's v_add_f32 /
v_mul_f32 round to nearest as numpy does)."""
import numpy as np


def test_idiv_f_exact():
    i = np.arange(4096, dtype=np.int64)
    for d in range(1, 730):
        r = np.float32(1.0) / np.float32(d)
        q = ((i.astype(np.float32) + np.float32(0.5)) * r).astype(np.int64)
        assert np.array_equal(q, i // d), d
