#!/usr/bin/env python3
"""Convert a gmsh 4.1 mesh (the reference's mesh/sphere.msh) into the coarse
arrays the sphere deck loads on machines without the reference checkout
(dealii-ns-gls_amd/data/sphere_coarse.npz): vertices, lexicographic hex
connectivity, boundary quads and their physical tags (glsmesh.read_msh).

    python scripts/convert_msh.py /root/reference/mesh/sphere.msh
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))
import glsmesh  # noqa: E402

src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/mesh/sphere.msh"
out = sys.argv[2] if len(sys.argv) > 2 else glsmesh.SPHERE_COARSE
c = glsmesh.read_msh(src)
np.savez_compressed(out, **c)
print(out, {k: v.shape for k, v in c.items()}, "boundary ids", sorted(set(c["bids"].tolist())))
