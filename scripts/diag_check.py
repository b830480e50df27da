import os, sys
sys.path[:0] = ['dealii-ns-gls_amd/python', 'oracle', 'tests']
import numpy as np, torch
import glsamd
from test_gpu_mg import _hierarchy, _np
from mg_ref import OracleGMG
from helpers import rel_err
for name, nref in [("input_turek_2D_Re20_stat.json", 2), ("input_hoffmann_3D_Re3900.json", 1)]:
    meshes, cmasks, params, w, u, hist = _hierarchy(name, nref)
    ref = OracleGMG(meshes, cmasks, params, u, hist, w)
    for mode in ("0", "1"):
        os.environ["GLS_DIAG_UNIT"] = mode
        mg, ops = glsamd.build_gmg(meshes, cmasks, params, u, hist, w, precision="f32")
        errs = []
        for l in range(len(meshes)):
            dl = ops[l].initialize_dof_vector(); ops[l].compute_inverse_diagonal(dl)
            d = _np(dl); r = ref.invdiag[l]
            i = np.argmax(np.abs(d - r) / np.abs(r))
            errs.append(f"l{l} rel_l2 {rel_err(d, r):.2e} worst {d[i]:.6g} vs {r[i]:.6g}")
        # FP64 level operators for comparison
        mg64, ops64 = glsamd.build_gmg(meshes, cmasks, params, u, hist, w, precision="f64")
        for l in range(len(meshes)):
            dl = ops64[l].initialize_dof_vector(); ops64[l].compute_inverse_diagonal(dl)
            errs.append(f"f64 l{l} {rel_err(_np(dl), ref.invdiag[l]):.2e}")
        print(name, "unit" if mode == "1" else "direct", "; ".join(errs), flush=True)
