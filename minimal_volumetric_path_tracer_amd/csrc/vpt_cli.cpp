/*
 * vpt_cli.cpp -- the `vpt` program: drop-in for the reference's `./rt <spp>` (src/rt.cpp:744-830).
 *
 *   vpt <spp> [--width W] [--height H] [--estimator ff|mis|explicit-free|implicit-free|explicit|surface-pt|ray-marching|ray-marching-sa|ray-marching-global|ray-marching-explicit] [--march-step S] [--march-light I] [--sigma-a A] [--sigma-s S]
 *             [--g G] [--max-depth D] [--seed N] [--device I] [--gpus N] [--fp64] [--out image.ppm]
 *
 * With only <spp> it renders the reference's default scene (include/Sphere.cpp:11-22), camera and
 * medium (src/rt.cpp:752-759,794) at 1024x768 with the free-flight estimator, writes image.ppm
 * in the reference's exact format and prints "elapsed time: <s>s" like src/rt.cpp:824-827.
 * --gpus N renders the image on devices 0 .. N-1 of this process (vpt_render_multi: interleaved
 * row bands, strips gathered over RCCL) -- the reference's OpenMP loop over all cores, at node
 * scale; the bytes are the same for any N.
 * Unlike the reference, a missing or bad argument is an error, not undefined behaviour.
 */
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "../../include/vpt.h"

static int usage()
{
    std::fprintf(stderr,
                 "usage: vpt <spp> [--width W] [--height H] [--estimator ff|mis|explicit-free|implicit-free|explicit|surface-pt|ray-marching|ray-marching-sa|ray-marching-global|ray-marching-explicit] [--march-step S] [--march-light I] [--sigma-a A] [--sigma-s S]\n"
                 "           [--g G] [--max-depth D] [--seed N] [--device I] [--gpus N] [--fp64] [--out image.ppm]\n");
    return 2;
}

int main(int argc, char** argv)
{
    if (argc < 2) return usage();
    auto start = std::chrono::system_clock::now();
    vpt_params p;
    vpt_default_params(&p);
    char* end = nullptr;
    long spp = std::strtol(argv[1], &end, 10);
    if (!end || *end || spp <= 0) return usage();
    p.spp = (int)spp;
    std::string out = "image.ppm";
    int device = 0, gpus = 0;
    for (int i = 2; i < argc; ++i) {
        std::string a = argv[i];
        auto need = [&](void) -> const char* {
            if (i + 1 >= argc) {
                usage();
                std::exit(2);
            }
            return argv[++i];
        };
        if (a == "--width") p.width = std::atoi(need());
        else if (a == "--height") p.height = std::atoi(need());
        else if (a == "--estimator") {
            std::string e = need();
            if (e == "ff") p.medium.estimator = VPT_FREE_FLIGHT;
            else if (e == "mis") p.medium.estimator = VPT_MIS_EQUIANGULAR;
            else if (e == "explicit-free") p.medium.estimator = VPT_EXPLICIT_FREE;
            else if (e == "implicit-free") p.medium.estimator = VPT_IMPLICIT_FREE;
            else if (e == "explicit") p.medium.estimator = VPT_EXPLICIT_EQUIANGULAR;
            else if (e == "surface-pt") p.medium.estimator = VPT_SURFACE_PT;
            else if (e == "ray-marching") p.medium.estimator = VPT_RAY_MARCHING;
            else if (e == "ray-marching-sa") p.medium.estimator = VPT_RAY_MARCHING_SA;
            else if (e == "ray-marching-global") p.medium.estimator = VPT_RAY_MARCHING_GLOBAL;
            else if (e == "ray-marching-explicit") p.medium.estimator = VPT_RAY_MARCHING_EXPLICIT;
            else return usage();
        } else if (a == "--march-step") p.medium.march_step = std::atof(need());
        else if (a == "--march-light") p.medium.march_light = std::atoi(need());
        else if (a == "--sigma-a") p.medium.sigma_a = std::atof(need());
        else if (a == "--sigma-s") p.medium.sigma_s = std::atof(need());
        else if (a == "--g") p.medium.hg_g = std::atof(need());
        else if (a == "--max-depth") p.medium.max_depth = std::atoi(need());
        else if (a == "--seed") p.seed = std::strtoull(need(), nullptr, 0);
        else if (a == "--device") device = std::atoi(need());
        else if (a == "--gpus") {
            gpus = std::atoi(need());
            if (gpus < 1) return usage();
        }
        else if (a == "--fp64") p.fb_format = VPT_FB_F64;
        else if (a == "--out") out = need();
        else return usage();
    }
    p.band_rows = p.height;
    std::vector<vpt_sphere> scene(VPT_MAX_SPHERES);
    int n = vpt_default_scene(scene.data(), (int)scene.size());
    vpt_context* ctx = nullptr;
    size_t elem = p.fb_format == VPT_FB_F64 ? sizeof(double) : sizeof(float);
    std::vector<char> fb((size_t)p.width * p.height * 3 * elem);
    int rc = VPT_OK;
    if (gpus > 0) {
        rc = vpt_render_multi(scene.data(), n, &p, gpus, fb.data());
    } else {
        rc = vpt_context_create(device, &ctx);
        if (rc == VPT_OK) rc = vpt_set_scene(ctx, scene.data(), n);
        if (rc == VPT_OK) rc = vpt_render(ctx, &p, fb.data());
    }
    if (rc == VPT_OK) rc = vpt_write_ppm(out.c_str(), fb.data(), p.fb_format, p.width, p.height);
    if (rc != VPT_OK) {
        std::fprintf(stderr, "vpt: error %d: %s\n", rc, vpt_last_error());
        vpt_context_destroy(ctx);
        return 1;
    }
    vpt_context_destroy(ctx);
    std::chrono::duration<double> elapsed = std::chrono::system_clock::now() - start;
    std::cout << "elapsed time: " << elapsed.count() << "s\n";
    return 0;
}
