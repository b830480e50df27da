// mg.hip — geometric multigrid (placeholder until the MG kernels land)
#include "../../include/gls_op.h"
#include "common.h"

struct glsMG_
{
};

extern "C" {
glsStatus gls_mg_create(const glsMGDesc *, const glsOp *, const uint32_t *const *, glsMG *)
{
  gls::set_error("gls_mg_create: not implemented yet");
  return 2;
}
void gls_mg_destroy(glsMG mg) { delete mg; }
glsStatus gls_mg_setup(glsMG, void *) { gls::set_error("not implemented"); return 2; }
glsStatus gls_mg_get_relaxation(glsMG, int, double *, double *) { gls::set_error("not implemented"); return 2; }
glsStatus gls_mg_vcycle(glsMG, void *, const void *, void *) { gls::set_error("not implemented"); return 2; }
glsStatus gls_mg_prolongate_add(glsMG, int, void *, const void *, void *) { gls::set_error("not implemented"); return 2; }
glsStatus gls_mg_restrict_add(glsMG, int, void *, const void *, void *) { gls::set_error("not implemented"); return 2; }
glsStatus gls_mg_interpolate(glsMG, int, void *, const void *, void *) { gls::set_error("not implemented"); return 2; }
glsStatus gls_mg_smooth(glsMG, int, void *, const void *, int, void *) { gls::set_error("not implemented"); return 2; }
}
