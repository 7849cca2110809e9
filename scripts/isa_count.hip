// Static instruction counts of the device functions on the hot path (one kernel per function).
// Build + count:  bash scripts/isa_count.sh
#include "../minimal_volumetric_path_tracer_amd/csrc/vpt_pool.h"

using namespace vpt;

#define IN3(p, k) mk(p[k], p[k + 1], p[k + 2])

extern "C" __global__ void k_sqrt(const double* in, double* out) { out[threadIdx.x] = vm_sqrt(in[threadIdx.x]); }
extern "C" __global__ void k_div(const double* in, double* out) { out[threadIdx.x] = in[threadIdx.x] / in[threadIdx.x + 1]; }
extern "C" __global__ void k_exp(const double* in, double* out) { out[threadIdx.x] = vm_exp(in[threadIdx.x]); }
extern "C" __global__ void k_log(const double* in, double* out) { out[threadIdx.x] = vm_log(in[threadIdx.x]); }
extern "C" __global__ void k_sincos(const double* in, double* out)
{
    double s, c;
    vm_sincos(in[threadIdx.x], &s, &c);
    out[threadIdx.x] = s + c;
}
extern "C" __global__ void k_acos(const double* in, double* out) { out[threadIdx.x] = vm_acos(in[threadIdx.x]); }
extern "C" __global__ void k_atan2(const double* in, double* out) { out[threadIdx.x] = vm_atan2(in[threadIdx.x], in[1]); }
extern "C" __global__ void k_tan(const double* in, double* out) { out[threadIdx.x] = vm_tan(in[threadIdx.x]); }
extern "C" __global__ void k_erand(uint64_t* X, double* out) { out[threadIdx.x] = vpt_erand48(&X[threadIdx.x]); }
extern "C" __global__ void k_stream(const uint64_t* in, uint64_t* out) { out[threadIdx.x] = vpt_stream_start(in[0], in[threadIdx.x], in[1]); }
extern "C" __global__ void k_nrm(const double* in, double* out)
{
    dv3 v = nrm(IN3(in, threadIdx.x));
    out[threadIdx.x] = v.x + v.y + v.z;
}
extern "C" __global__ void k_intersect(const DevScene* S, const double* in, double* out)
{
    Sampler<false> smp;
    smp.X = 1;
    double t;
    int id = 0;
    scene_intersect(S, smp, IN3(in, threadIdx.x), IN3(in, threadIdx.x + 3), t, id, false);
    out[threadIdx.x] = t + id;
}
extern "C" __global__ void k_solid_angle_dir(const double* in, double* out, uint64_t* X)
{
    Sampler<false> smp;
    smp.X = X[threadIdx.x];
    dv3 v = solid_angle_dir(smp, IN3(in, threadIdx.x), in[threadIdx.x + 3]);
    out[threadIdx.x] = v.x + v.y + v.z;
}
extern "C" __global__ void k_fr_microfacet(const double* in, double* out)
{
    dv3 v = fr_microfacet(IN3(in, 0), IN3(in, 3), IN3(in, threadIdx.x), IN3(in, threadIdx.x + 3), IN3(in, threadIdx.x + 6),
                          in[1], IN3(in, threadIdx.x + 9));
    out[threadIdx.x] = v.x + v.y + v.z;
}
extern "C" __global__ void k_vector_facet(const double* in, double* out, uint64_t* X)
{
    Sampler<false> smp;
    smp.X = X[threadIdx.x];
    dv3 v = vector_facet(smp, in[0]);
    out[threadIdx.x] = v.x + v.y + v.z;
}
template <int EST, int which>
__device__ __forceinline__ void run_stage( const DevScene* S, double* in, double* out, uint64_t* X)
{
    Sampler<false> smp;
    smp.X = X[threadIdx.x];
    smp.g = in[100];
    Medium m{in[101], in[102], in[103], (int)in[104]};
    Path p;
    p.o = IN3(in, threadIdx.x);
    p.d = IN3(in, threadIdx.x + 3);
    p.beta = IN3(in, threadIdx.x + 6);
    p.L = IN3(in, threadIdx.x + 9);
    p.depth = (int)in[threadIdx.x + 12];
    Event e;
    e.t = in[threadIdx.x + 13];
    e.dist = in[threadIdx.x + 14];
    e.pdf = in[threadIdx.x + 15];
    e.id = (int)in[threadIdx.x + 16];
    e.src = (int)in[threadIdx.x + 17];
    int r = 0;
    if (which == 0) r = decide<EST>(S, smp, p, e, m);
    else if (which == 1) surface_event<EST>(S, smp, p, e, m);
    else medium_event<EST>(S, smp, p, e, m);
    out[threadIdx.x] = p.L.x + p.L.y + p.beta.z + p.d.x + p.o.y + e.dist + r;
    X[threadIdx.x] = smp.X;
}
extern "C" __global__ void k_decide_ff(const DevScene* S, double* in, double* out, uint64_t* X) { run_stage<0, 0>(S, in, out, X); }
extern "C" __global__ void k_surface_ff(const DevScene* S, double* in, double* out, uint64_t* X) { run_stage<0, 1>(S, in, out, X); }
extern "C" __global__ void k_medium_ff(const DevScene* S, double* in, double* out, uint64_t* X) { run_stage<0, 2>(S, in, out, X); }
extern "C" __global__ void k_decide_mis(const DevScene* S, double* in, double* out, uint64_t* X) { run_stage<1, 0>(S, in, out, X); }
extern "C" __global__ void k_surface_mis(const DevScene* S, double* in, double* out, uint64_t* X) { run_stage<1, 1>(S, in, out, X); }
extern "C" __global__ void k_medium_mis(const DevScene* S, double* in, double* out, uint64_t* X) { run_stage<1, 2>(S, in, out, X); }
extern "C" __global__ void k_p_light(const DevScene* S, double* in, double* out, uint64_t* X)
{
    Sampler<false> smp;
    smp.X = X[threadIdx.x];
    dv3 v = p_light(S, smp, (int)in[0], IN3(in, threadIdx.x), IN3(in, threadIdx.x + 3), IN3(in, threadIdx.x + 6),
                    (int)in[1], in[2]);
    out[threadIdx.x] = v.x + v.y + v.z;
}
extern "C" __global__ void k_mis_v2(const DevScene* S, double* in, double* out, uint64_t* X)
{
    Sampler<false> smp;
    smp.X = X[threadIdx.x];
    dv3 v = mis_v2(S, smp, (int)in[0], IN3(in, threadIdx.x), IN3(in, threadIdx.x + 3), IN3(in, threadIdx.x + 6), in[2], in[3]);
    out[threadIdx.x] = v.x + v.y + v.z;
}
extern "C" __global__ void k_bdsf(const DevScene* S, double* in, double* out, uint64_t* X)
{
    Sampler<false> smp;
    smp.X = X[threadIdx.x];
    dv3 aux;
    double prob;
    dv3 v = bdsf(S, smp, aux, IN3(in, threadIdx.x), IN3(in, threadIdx.x + 3), prob, (int)in[0]);
    out[threadIdx.x] = v.x + v.y + v.z + aux.x + prob;
}
extern "C" __global__ void k_single_scattering(const DevScene* S, double* in, double* out, uint64_t* X)
{
    Sampler<false> smp;
    smp.X = X[threadIdx.x];
    smp.g = in[5];
    dv3 v = single_scattering(S, smp, IN3(in, threadIdx.x), IN3(in, threadIdx.x + 3), (int)in[0], in[1], false, in[2],
                              1.0, in[3]);
    out[threadIdx.x] = v.x + v.y + v.z;
}
extern "C" __global__ void k_phase_sample(double* in, double* out, uint64_t* X)
{
    Sampler<false> smp;
    smp.X = X[threadIdx.x];
    smp.g = in[5];
    dv3 v = phase_sample(smp, IN3(in, threadIdx.x));
    out[threadIdx.x] = v.x + v.y + v.z;
}

/* specialised stage bodies as the pool kernel instantiates them */
template <int MK, int PT>
__device__ __forceinline__ void run_surface(const DevScene* S, double* in, double* out, uint64_t* X)
{
    Sampler<false> smp;
    smp.X = X[threadIdx.x];
    smp.g = in[100];
    Medium m{in[101], in[102], in[103], (int)in[104]};
    Path p;
    p.o = IN3(in, threadIdx.x);
    p.d = IN3(in, threadIdx.x + 3);
    p.beta = IN3(in, threadIdx.x + 6);
    p.L = IN3(in, threadIdx.x + 9);
    p.depth = (int)in[threadIdx.x + 12];
    Event e;
    e.t = in[threadIdx.x + 13];
    e.dist = in[threadIdx.x + 14];
    e.pdf = in[threadIdx.x + 15];
    e.id = (int)in[threadIdx.x + 16];
    e.src = (int)in[threadIdx.x + 17];
    surface_event<0, false, MK, PT>(S, smp, p, e, m);
    out[threadIdx.x] = p.L.x + p.L.y + p.beta.z + p.d.x + p.o.y;
    X[threadIdx.x] = smp.X;
}
extern "C" __global__ void k_surface_diffuse_sphere(const DevScene* S, double* in, double* out, uint64_t* X) { run_surface<0, 0>(S, in, out, X); }
extern "C" __global__ void k_surface_diffuse_point(const DevScene* S, double* in, double* out, uint64_t* X) { run_surface<0, 1>(S, in, out, X); }
extern "C" __global__ void k_mis_v2_diffuse(const DevScene* S, double* in, double* out, uint64_t* X)
{
    Sampler<false> smp;
    smp.X = X[threadIdx.x];
    dv3 v = mis_v2<false, 0>(S, smp, (int)in[0], IN3(in, threadIdx.x), IN3(in, threadIdx.x + 3), IN3(in, threadIdx.x + 6), in[2], in[3]);
    out[threadIdx.x] = v.x + v.y + v.z;
}
extern "C" __global__ void k_p_light_diffuse(const DevScene* S, double* in, double* out, uint64_t* X)
{
    Sampler<false> smp;
    smp.X = X[threadIdx.x];
    dv3 v = p_light<false, 0, 0>(S, smp, (int)in[0], IN3(in, threadIdx.x), IN3(in, threadIdx.x + 3), IN3(in, threadIdx.x + 6),
                                 (int)in[1], in[2]);
    out[threadIdx.x] = v.x + v.y + v.z;
}
extern "C" __global__ void k_bdsf_diffuse(const DevScene* S, double* in, double* out, uint64_t* X)
{
    Sampler<false> smp;
    smp.X = X[threadIdx.x];
    dv3 aux;
    double prob;
    dv3 v = bdsf<false, 0>(S, smp, aux, IN3(in, threadIdx.x), IN3(in, threadIdx.x + 3), prob, (int)in[0]);
    out[threadIdx.x] = v.x + v.y + v.z + aux.x + prob;
}
extern "C" __global__ void k_medium_sphere(const DevScene* S, double* in, double* out, uint64_t* X)
{
    Sampler<false> smp;
    smp.X = X[threadIdx.x];
    smp.g = in[100];
    Medium m{in[101], in[102], in[103], (int)in[104]};
    Path p;
    p.o = IN3(in, threadIdx.x);
    p.d = IN3(in, threadIdx.x + 3);
    p.beta = IN3(in, threadIdx.x + 6);
    p.L = IN3(in, threadIdx.x + 9);
    p.depth = 0;
    Event e;
    e.dist = in[threadIdx.x + 14];
    e.src = (int)in[threadIdx.x + 17];
    medium_event<0, false, 0>(S, smp, p, e, m);
    out[threadIdx.x] = p.L.x + p.L.y + p.beta.z + p.d.x + p.o.y;
    X[threadIdx.x] = smp.X;
}
