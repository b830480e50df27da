"""constraints_inhomogeneous (main.cc:879-891): the host generator of the
inflow Dirichlet values (glsmesh.Deck.constraint_values) against the closed
form of InflowBoundaryValues::Channel (simulation.cc:25-76) and the
constraint structure (values only on constrained components that
constraints_copy leaves free).  CPU only."""
import numpy as np

from helpers import deck


def _setup(name, n_ref, **over):
    d = deck(name)
    for k, v in over.items():
        setattr(d, k, v)
    m = d.mesh(n_ref)
    vel, p, slip = d.boundary_descriptor()
    return d, m, m.constraint_mask(vel, p, slip)


def test_re3900_uniform_inflow():
    d, m, cm = _setup("input_hoffmann_3D_Re3900.json", 1)
    g = d.constraint_values(m, t=0.0)
    nc = m.dim + 1
    inflow = np.nonzero(m.node_boundary & 1)[0]
    # slip walls constrain only the normal component: every inflow node's
    # x velocity is an inhomogeneous Dirichlet dof with the value u_max
    assert np.all(g[inflow * nc] == d.u_max)
    nz = np.nonzero(g)[0]
    assert nz.size == inflow.size
    assert np.all(((cm[nz // nc] >> (nz % nc)) & 1) == 1)
    assert np.all(nz % nc == 0)


def test_parabolic_profile_and_ramp():
    d, m, cm = _setup("input_hoffmann_3D_Re3900.json", 1, no_slip_wall=True, t_init=0.5)
    H = m.params["height"]
    g = d.constraint_values(m, t=0.25)
    nc = m.dim + 1
    nodes = np.nonzero(g)[0] // nc
    x = m.coords[nodes]
    y = x[:, 1] + H / 2.0 - d.cylinder_shift
    z = x[:, 2] + H / 2.0
    expect = 0.5 * d.u_max * (4 * y * (H - y) / H / H) * (4 * z * (H - z) / H / H)
    assert np.allclose(g[nodes * nc], expect, rtol=1e-14, atol=0)
    # no-slip walls own the inflow edges: those dofs stay homogeneous
    walls = ((m.node_boundary >> 3) & 0x3F) != 0
    edge = np.nonzero((m.node_boundary & 1).astype(bool) & walls)[0]
    assert edge.size > 0 and np.all(g[edge * nc] == 0)
    assert abs(d.constraint_values(m, t=1.0).max() - d.u_max) < 0.05 * d.u_max


def test_2d_deck():
    d, m, cm = _setup("input_turek_2D_Re100.json", 2)
    # the deck ramps the inflow up over t_init = 0.01: zero at t = 0
    assert not d.constraint_values(m, t=0.0).any()
    g = d.constraint_values(m, t=0.02)
    nc = m.dim + 1
    nz = np.nonzero(g)[0]
    assert nz.size > 0 and np.all(nz % nc == 0)
    assert np.all(((cm[nz // nc] >> 0) & 1) == 1)
    assert g.max() <= d.u_max * (1 + 1e-12) and g.max() > 0.95 * d.u_max
