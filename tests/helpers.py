"""Shared setup for parity tests: one deck-like configuration -> mesh,
constraint mask, operator parameters and the §8d synthetic inputs, plus the
oracle (TEST INFRASTRUCTURE) on the same data."""
import numpy as np

import glsinputs as gi
import glsmesh as gm
import oracle as orc

DECKS = ["input_turek_2D_Re20_stat.json", "input_turek_2D_Re100.json",
         "input_turek_3D_Re100.json", "input_hoffmann_3D_Re3900.json"]


def deck(name):
    return gm.read_deck(f"{gm.DECK_DIR}/{name}")


class Case:
    def __init__(self, mesh, cmask, params, weights, u_inf=1.0, seed_shift=0):
        self.mesh, self.cmask, self.params, self.weights = mesh, cmask, params, weights
        self.dim = mesh.dim
        self.n_dofs = mesh.n_dofs
        self.src = gi.src_vector(self.n_dofs)
        self.u_star = gi.linearization_point(mesh.n_nodes, mesh.dim, u_inf)
        self.hist = gi.history(self.u_star, params["order"])

    def oracle(self, outflow=None):
        om = orc.OracleMesh(self.mesh, self.cmask)
        o = orc.Oracle(om, **self.params)
        if outflow is not None:
            o.set_outflow_faces(*outflow)
        o.set_linearization_point(self.u_star)
        if self.params["order"] > 0:
            o.set_previous_solution(self.hist, self.weights)
        self._om = om
        return o

    def gpu(self, precision="f64", brick=None, outflow=None):
        import glsamd
        op = glsamd.NavierStokesOperator(self.mesh, self.cmask, precision, brick=brick,
                                         outflow=outflow)
        op.set_parameters(**self.params)
        op.set_linearization_point(self.u_star)
        if self.params["order"] > 0:
            op.set_previous_solution(self.hist, self.weights)
        return op


def deck_case(name, n_ref=None, dt=2.5e-4, **overrides):
    d = deck(name)
    for k, v in overrides.items():
        setattr(d, k, v)
    m = d.mesh(n_ref)
    vel, p, slip = d.boundary_descriptor()
    cmask = m.constraint_mask(vel, p, slip)
    params, w = d.operator_parameters(dt)
    return Case(m, cmask, params, w, u_inf=d.u_max)


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)
