// gs_phys_inst.hip -- explicit instantiation of ONE physics kernel form for ONE topology.
// Compiled once per (topology, form) by isaacgymenv_amd/build.py with
//   -DGS_INST_TOPO=Topo_<name> -DGS_INST_FORM=<0 sim plane | 1 sim terrain | 2 pd plane | 3 pd terrain>
// so that the solver instantiations (UsefulHound's take minutes each) compile in parallel.
#include "gs_physics_impl.h"

#if !defined(GS_INST_TOPO) || !defined(GS_INST_FORM)
#error "gs_phys_inst.hip is compiled by isaacgymenv_amd/build.py with GS_INST_TOPO and GS_INST_FORM"
#endif

#if GS_INST_FORM == 0
template hipError_t launch_sim_plane<GS_INST_TOPO>(const DevModel*, const DevParams&, const SimBuffers&, const float*,
                                                   hipStream_t);
template hipError_t launch_dbg_pool<GS_INST_TOPO>(const DevModel*, const DevParams&, const SimBuffers&, int, float*,
                                                  int*, hipStream_t);
#elif GS_INST_FORM == 1
template hipError_t launch_sim_terr<GS_INST_TOPO>(const DevModel*, const DevParams&, const SimBuffers&, const float*,
                                                  hipStream_t);
#elif GS_INST_FORM == 2
template hipError_t launch_pd_plane<GS_INST_TOPO>(const DevModel*, const DevParams&, const SimBuffers&, const PdDev&,
                                                  hipStream_t);
#else
template hipError_t launch_pd_terr<GS_INST_TOPO>(const DevModel*, const DevParams&, const SimBuffers&, const PdDev&,
                                                 hipStream_t);
#endif

#ifdef GS_PHASE_PROFILE
// the wave-assisted kernels' phase cycles of this translation unit (gs_physics_impl.h gs_wave_cycles)
#define GS_WCAT2(a, b, c) a##b##_##c
#define GS_WCAT(a, b, c) GS_WCAT2(a, b, c)
extern "C" __attribute__((visibility("default"))) int GS_WCAT(gs_debug_wave_cycles_, GS_INST_TOPO, GS_INST_FORM)(
    unsigned long long* out, int n, int reset) {
  if (n > 16) n = 16;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gs_phys::gs_wave_cycles), n * sizeof(unsigned long long)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(gs_phys::gs_wave_cycles), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif
