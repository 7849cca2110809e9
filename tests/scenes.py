"""Scenes used by the parity fixtures and tests (numpy records with the reference Sphere layout,
include/Sphere.h:12-21, 144 bytes).  `default` is include/Sphere.cpp:11-22; the others widen
coverage to branches the default scene never takes."""
import numpy as np

SPHERE_DTYPE = np.dtype(
    {
        "names": ["r", "p", "c", "radiance", "material", "reserved_", "eta", "kappa", "alpha"],
        "formats": ["<f8", ("<f8", 3), ("<f8", 3), ("<f8", 3), "<i4", "<i4", ("<f8", 3), ("<f8", 3), "<f8"],
        "offsets": [0, 8, 32, 56, 80, 84, 88, 112, 136],
        "itemsize": 144,
    }
)

AL_ETA = (1.66058, 0.88143, 0.521467)
AL_KAPPA = (9.2282, 6.27077, 4.83803)


def sph(r, p, c=(0, 0, 0), rad=(0, 0, 0), mat=0, eta=(0, 0, 0), kappa=(0, 0, 0), alpha=0.0):
    s = np.zeros(1, dtype=SPHERE_DTYPE)
    s["r"], s["p"], s["c"], s["radiance"], s["material"] = r, p, c, rad, mat
    s["eta"], s["kappa"], s["alpha"] = eta, kappa, alpha
    return s


def walls(left=(.5, .5, .5), right=(.0, .0, .5)):
    return [
        sph(1e5, (-1e5 - 49, 0, 0), left),
        sph(1e5, (1e5 + 49, 0, 0), right),
        sph(1e5, (0, 0, -1e5 - 81.6), (.5, .5, .5)),
        sph(1e5, (0, -1e5 - 40.8, 0), (.5, .5, .5)),
        sph(1e5, (0, 1e5 + 40.8, 0), (.5, .5, .5)),
    ]


def default_scene():
    return np.concatenate(walls() + [
        sph(16.5, (-23, -24.3, -34.6), mat=1, eta=AL_ETA, kappa=AL_KAPPA, alpha=0.09),
        sph(16.5, (23, -24.3, -3.6), (.0, .0, .9)),
        sph(2, (0, 24.3, -35), rad=(100, 100, 0)),
        sph(0, (-23, 24.3, 0), rad=(6000, 0, 0)),
        sph(2, (23, 24.3, 35), rad=(75, 75, 60)),
    ])


def dielectric_scene():
    """blue Lambert sphere replaced by a smooth dielectric (material 2, eta 1.5 hard-coded)."""
    s = default_scene()
    s[6]["material"] = 2
    s[6]["c"] = (.9, .9, .9)
    return s


def mat3_scene():
    """a material-3 ("volumetric") sphere around the point light: shadow rays fall back to
    visibilityVPT + multipleT (include/vptShadeMethods.h:68-72)."""
    return np.concatenate([default_scene(), sph(4.0, (-23, 24.3, 0), (.5, .5, .5), mat=3)])


def point_lights_scene():
    """only point lights: the MISv2 light loop is empty (include/misSamplingFunctions.h:106)."""
    return np.concatenate(walls() + [
        sph(16.5, (-23, -24.3, -34.6), mat=1, eta=AL_ETA, kappa=AL_KAPPA, alpha=0.3),
        sph(16.5, (23, -24.3, -3.6), (.7, .6, .2)),
        sph(0, (-23, 24.3, 0), rad=(3000, 3000, 1000)),
        sph(0, (20, 10, -40), rad=(1000, 2000, 4000)),
    ])


def no_emitter_scene():
    s = default_scene()
    return np.concatenate([s[:7]])


def big_light_scene():
    """default scene with an emissive ceiling (a 1e5-radius emitter): paths hit a light often, so
    the implicit estimator (which only scores on a light hit) is exercised."""
    s = default_scene()
    s[4]["radiance"] = (4.0, 4.0, 3.0)
    return s


SCENES = {
    "default": default_scene,
    "dielectric": dielectric_scene,
    "mat3": mat3_scene,
    "point_lights": point_lights_scene,
    "no_emitter": no_emitter_scene,
}

# scenes of the estimator fixtures (tests/golden/samples_e234.npz)
EST_SCENES = dict(SCENES, big_light=big_light_scene)

# ---- the reference's alternate scenes (commented out in include/Sphere.cpp), as parity cases
AL2_ETA, AL2_KAPPA = (0.143245, 0.377423, 1.43919), (3.98479, 2.3847, 1.60434)


def alt_metal_walls_scene():
    """include/Sphere.cpp:27-45 ("escena dos"): conductor side walls, coloured box, one point light."""
    return np.concatenate([
        sph(1e5, (-1e5 - 49, 0, 0), mat=1, eta=AL_ETA, kappa=AL_KAPPA, alpha=0.03),
        sph(1e5, (1e5 + 49, 0, 0), mat=1, eta=AL_ETA, kappa=AL_KAPPA, alpha=0.03),
        sph(1e5, (0, 0, -1e5 - 81.6), (.25, .75, .25)),
        sph(1e5, (0, -1e5 - 40.8, 0), (.25, .75, .75)),
        sph(1e5, (0, 1e5 + 40.8, 0), (.75, .75, .25)),
        sph(16.5, (-23, -24.3, -34.6), (.75, .75, .25)),
        sph(16.5, (23, -24.3, -3.6), (.4, .3, .2)),
        sph(0, (14, -24.3, -35), rad=(2000, 2000, 3000)),
    ])


def alt_light_near_camera_scene():
    """include/Sphere.cpp:47-60 ("escena 3"): no walls, two spheres and a point light right in
    front of the camera."""
    return np.concatenate([
        sph(30, (0, 11.2, 165), (.0, .25, .75)),
        sph(16.5, (0, -10, 200), (.75, .75, .75)),
        sph(0, (0, 11.2, 204), rad=(400, 400, 400)),
    ])


def alt_area_light_scene():
    """include/Sphere.cpp:62-74: coloured box without ceiling, conductor sphere, one r=12 area light."""
    return np.concatenate([
        sph(1e5, (-1e5 - 49, 0, 0), (.75, .25, .25)),
        sph(1e5, (1e5 + 49, 0, 0), (.25, .25, .75)),
        sph(1e5, (0, 0, -1e5 - 81.6), (.25, .75, .25)),
        sph(1e5, (0, -1e5 - 40.8, 0), (.25, .75, .75)),
        sph(16.5, (-23, -24.3, -34.6), mat=1, eta=AL_ETA, kappa=AL_KAPPA, alpha=0.03),
        sph(12, (24, 24.3, -50), rad=(0, 800, 800)),
    ])


def alt_open_space_scene():
    """include/Sphere.cpp:76-86 ("primitive infinite"): no walls, conductor spheres floating in the
    medium, three point lights -- rays escape (t = MAXFLOAT paths)."""
    return np.concatenate([
        sph(16.5, (-23, -24.3, -34.6), mat=1, eta=AL_ETA, kappa=AL_KAPPA, alpha=0.03),
        sph(16.5, (23, -24.3, -3.6), mat=1, eta=AL2_ETA, kappa=AL2_KAPPA, alpha=0.3),
        sph(100, (0, -24.3, -200), mat=1, eta=AL2_ETA, kappa=AL2_KAPPA, alpha=0.02),
        sph(0, (24, 24.3, -3.6), rad=(2000, 2000, 2000)),
        sph(0, (-24, 10, -34.6), rad=(2000, 5000, 1000)),
        sph(0, (0, -24.3, -30), rad=(4000, 8000, 4000)),
    ])


def alt_point_box_scene():
    """include/Sphere.cpp:88-105: grey box, one Lambert sphere, two point lights."""
    return np.concatenate(walls((.5, .5, .5), (.5, .5, .5)) + [
        sph(16.5, (23, -24.3, -3.6), (.50, .50, 0)),
        sph(0, (-23, 0, -10.6), (1, 1, 1), rad=(6000, 6000, 6000)),
        sph(0, (23, 24.3, -50), (1, 1, 1), rad=(4000, 4000, 4000)),
    ])


ALT_SCENES = {
    "alt_metal_walls": alt_metal_walls_scene,
    "alt_light_near_camera": alt_light_near_camera_scene,
    "alt_area_light": alt_area_light_scene,
    "alt_open_space": alt_open_space_scene,
    "alt_point_box": alt_point_box_scene,
}


# independent (pure Python) statement of the per-sample stream spec (csrc/vpt_rng.h)
M64 = (1 << 64) - 1


def splitmix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def stream_state(seed, idx, sample):
    k = splitmix64((seed + 0x9E3779B97F4A7C15 * (idx + 1)) & M64)
    return splitmix64(k ^ ((sample * 0xD1B54A32D192ED03 + 1) & M64)) >> 16
