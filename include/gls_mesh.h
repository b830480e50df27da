/*
 * gls_mesh.h — C-ABI of the host-side mesh / DoF / constraint setup library
 * (libglsmesh.so, plain C++, no GPU).
 *
 * In the reference this work is done by deal.II before the operator is
 * built: the triangulation (`cylinder()` grid_cylinder.h:7-242, refined in
 * SimulationCylinder::create_triangulation simulation.cc:300-376), the
 * DoFHandler for FESystem(FE_Q(k), dim+1) (main.cc:239-242), the MappingQ_k
 * support points (main.cc:251-256) and the AffineConstraints built from the
 * boundary descriptor (main.cc:259-310, simulation.cc:378-431).  This library
 * restates exactly the part of that pipeline the hot path consumes:
 *
 *   - a refined hex/quad mesh in which every cell lists its (k+1)^dim Q_k
 *     support points ("nodes") in lexicographic order,
 *   - node coordinates (the MappingQ_k support points; mapping degree == fe
 *     degree as in every target deck, "mapping degree": 0 → fe degree),
 *   - per-node boundary-id bitmasks and the per-node constrained-component
 *     mask for a boundary descriptor,
 *   - the parent→child node lattice between consecutive geometric levels
 *     (what MGTwoLevelTransfer needs, main.cc:538-563).
 *
 * DoF numbering (our choice, not part of the parity contract — SURVEY §8e):
 *   dof = node * (dim + 1) + component,  component dim == pressure.
 */
#ifndef GLS_MESH_H
#define GLS_MESH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct glsMesh_ glsMesh;

/* Boundary ids follow grid_cylinder.h:112-133 / :200-223:
 *   0 inflow, 1 outflow, 2 cylinder, 3/4 y-walls (bottom/top), 5/6 z-walls. */
enum { GLS_BID_INFLOW = 0, GLS_BID_OUTFLOW = 1, GLS_BID_CYLINDER = 2 };

/* Flow-past-cylinder channel (grid_cylinder.h:7-242): dim = 2 or 3,
 * degree k in {1,2}, n_ref global refinements.  For dim == 3 the 2D
 * cross-section is built with for_3D = true (4 columns upstream) and
 * extruded into 4 layers of height `height` centred at z = 0.
 * Returns 0 on success. */
int gls_mesh_cylinder(int dim, int degree, int n_ref, double length,
                      double height, double cylinder_position,
                      double cylinder_diameter, double shift, glsMesh **out);

/* Unit hyper cube [0,1]^dim refined n_ref times (performance.cc:28-31);
 * degree k in {1,2,3}; every boundary face has id 0. */
int gls_mesh_hypercube(int dim, int degree, int n_ref, glsMesh **out);

/* An unstructured coarse hex (quad) mesh refined n_ref times — the sphere
 * deck's GridIn::read_msh + refine_global (simulation.cc:858-872).
 * cells: [n_cells][2^dim] vertex indices in lexicographic order (x fastest;
 * gmsh's hexahedron order 0 1 2 3 4 5 6 7 maps to 0 1 3 2 4 5 7 6);
 * boundary elements: [n_bfaces][2^(dim-1)] vertex indices with their
 * physical tags (the boundary ids; untagged boundary faces get 0).
 * Refinement is flat (multilinear): SphericalManifold is attached to
 * manifold id 0, which read_msh leaves unset on every object, so it
 * bends nothing — parity unpinned, see DESIGN.md.  degree k in {1,2}. */
int gls_mesh_from_coarse(int dim, int degree, int n_ref, int64_t n_vertices,
                         const double *vertices, int64_t n_cells,
                         const int32_t *cells, int64_t n_bfaces,
                         const int32_t *bface_vertices,
                         const int32_t *bface_ids, glsMesh **out);

void gls_mesh_destroy(glsMesh *m);

int     gls_mesh_dim(const glsMesh *m);
int     gls_mesh_degree(const glsMesh *m);
int64_t gls_mesh_n_cells(const glsMesh *m);
int64_t gls_mesh_n_nodes(const glsMesh *m);
int64_t gls_mesh_n_coarse_cells(const glsMesh *m);

/* [n_cells * (k+1)^dim] node indices, lexicographic (x fastest). */
const uint32_t *gls_mesh_cell_nodes(const glsMesh *m);
/* [n_nodes * dim] node coordinates. */
const double *gls_mesh_node_coords(const glsMesh *m);
/* [n_nodes] bit b set <=> node lies on a boundary face with id b. */
const uint32_t *gls_mesh_node_boundary(const glsMesh *m);
/* [n_cells] index of the coarse cell the fine cell descends from. */
const int32_t *gls_mesh_cell_coarse(const glsMesh *m);

/* Per-node constrained-component mask (bit c = component c constrained to
 * zero) for the boundary descriptor:
 *   vel_ids   bitmask of ids with homogeneous velocity Dirichlet
 *             (all_homogeneous_dbcs + all_inhomogeneous_dbcs made zero,
 *              main.cc:265-291),
 *   p_ids     bitmask of ids with zero pressure (all_homogeneous_nbcs,
 *             main.cc:271-275),
 *   slip_ids  bitmask of ids with no-normal-flux on axis-aligned planar
 *             walls (main.cc:277-279); ids 3/4 constrain u_y, 5/6 u_z.
 * out has n_nodes entries.  Returns 0 on success. */
int gls_mesh_constraint_mask(const glsMesh *m, uint32_t vel_ids,
                             uint32_t p_ids, uint32_t slip_ids,
                             uint8_t *out);

/* Cells are ordered brick-major inside every coarse cell: bricks of
 * dims[0] x dims[1] x dims[2] cells (min(2^n_ref, 4) per direction in 3D,
 * min(2^n_ref, 8) in 2D), lexicographic inside a brick, so the cell list is
 * a sequence of equal-shape bricks — the structure hint glsOpDesc.brick
 * takes.  Returns 0 on success. */
int gls_mesh_brick(const glsMesh *m, int *dims);

/* Child lattice for MG transfer: `coarse` and `fine` must come from the same
 * generator call parameters with fine.n_ref == coarse.n_ref + 1.  For every
 * coarse-level cell, writes the (2k+1)^dim fine-level node indices of the
 * lattice covering its 2^dim children (lexicographic).  out has
 * n_cells(coarse) * (2k+1)^dim entries.  Returns 0 on success. */
int gls_mesh_child_lattice(const glsMesh *coarse, const glsMesh *fine,
                           uint32_t *out);

/* Vertex-based cell measure (deal.II cell->measure(): area of the bilinear
 * quad / volume of the trilinear hex through the 2^dim vertices, used by
 * compute_penalty_parameters operator_ns.cc:399) and the minimum vertex
 * distance (operator_ns.cc:374), per cell. */
int gls_mesh_cell_measure(const glsMesh *m, double *measure_out,
                          double *min_vertex_distance_out);

const char *gls_mesh_last_error(void);

#ifdef __cplusplus
}
#endif

#endif
