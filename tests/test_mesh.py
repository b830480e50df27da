"""Mesh / DoF / constraint setup (libglsmesh.so) against the reference's
counts (main.cc:246-249 prints them) and structural properties."""
import numpy as np
import pytest

import glsmesh as gm
from helpers import deck


@pytest.mark.parametrize("name,cells,dofs", [
    ("input_turek_2D_Re20_stat.json", 1408, 17592),
    ("input_turek_2D_Re100.json", 90112, 273120),
    ("input_hoffmann_3D_Re3900.json", 25600, 878592),
])
def test_deck_counts(name, cells, dofs):
    m = deck(name).mesh()
    assert (m.n_cells, m.n_dofs) == (cells, dofs)


def test_turek_3d_counts():
    # input_turek_3D_Re100.json: same mesh family at r3
    m = deck("input_turek_3D_Re100.json").mesh()
    assert (m.n_cells, m.n_dofs) == (204800, 6789120)


def test_coarse_mesh():
    # grid_cylinder.h: 100 coarse quads in the 3D cross section -> 400 hexes,
    # 88 quads in 2D
    assert gm.cylinder(3, 1, 0).n_cells == 400
    assert gm.cylinder(2, 1, 0).n_cells == 88
    assert gm.cylinder(3, 1, 0).n_nodes == 660  # coarse vertices V
    assert gm.cylinder(2, 1, 0).n_nodes == 117


@pytest.mark.parametrize("dim", [2, 3])
def test_geometry(dim):
    m = gm.cylinder(dim, 2, 1)
    meas, hmin = m.cell_measure()
    assert (meas > 0).all() and (hmin > 0).all()
    H, L = 0.41, (2.2 if dim == 2 else 2.5)
    exact = (L * H - np.pi * 0.05 ** 2) * (H if dim == 3 else 1)
    assert abs(meas.sum() - exact) / exact < 1e-3
    # cylinder nodes sit on the cylinder surface (manifold id 0)
    on = (m.node_boundary >> 2) & 1
    r = np.hypot(m.coords[on == 1, 0], m.coords[on == 1, 1])
    assert np.allclose(r, 0.05, atol=1e-14)


def test_nested_levels():
    c, f = gm.cylinder(3, 2, 1, shift=0.0), gm.cylinder(3, 2, 2, shift=0.0)
    lat = c.child_lattice(f)
    assert lat.shape == (c.n_cells, 125)
    sel = [i + 5 * (j + 5 * l) for l in (0, 2, 4) for j in (0, 2, 4) for i in (0, 2, 4)]
    assert np.array_equal(f.coords[lat[:, sel]], c.coords[c.cell_nodes])


def test_constraint_masks_re3900():
    d = deck("input_hoffmann_3D_Re3900.json")
    m = d.mesh(0)
    vel, p, slip = d.boundary_descriptor()
    assert vel == [0, 2] and p == [1] and slip == [3, 4, 5, 6, 7, 8]
    mask = m.constraint_mask(vel, p, slip)
    b = m.node_boundary
    inflow, outflow, cyl = (b & 1) > 0, (b & 2) > 0, (b & 4) > 0
    ywall, zwall = (b & (8 | 16)) > 0, (b & (32 | 64)) > 0
    assert ((mask[inflow | cyl] & 7) == 7).all()
    assert ((mask[ywall] >> 1) & 1).all()
    assert ((mask[zwall] >> 2) & 1).all()
    assert (((mask >> 3) & 1) == outflow).all()
    interior = b == 0
    assert (mask[interior] == 0).all()


def test_curved_slip_rejected():
    m = gm.cylinder(3, 1, 0)
    with pytest.raises(RuntimeError, match="not an axis-aligned"):
        m.constraint_mask([], [], [2])  # slip on the cylinder: not a pure mask


def test_hypercube():
    m = gm.hypercube(3, 2, 2)
    assert m.n_cells == 64 and m.n_nodes == 9 ** 3
    meas, _ = m.cell_measure()
    assert abs(meas.sum() - 1) < 1e-14
