"""Adversarial scenes for the vertex kernel's two exactness shortcuts, against the oracle.

* The light-plane skip: a shadow ray meeting the light at |cos| >= 0.25 skips the candidates that lie
  within eta = 0.0015 of the sampled light triangle's plane, parallel to it (|cos| >= 0.999) and not
  slivers (rt_scene.cpp; MC/Renderer.cpp:172-189).  Scene A puts small tilted quads at 0.5, 0.9 and 0.99
  eta below the light (between the shaded points and the light: the reference blocks through them only
  at |cos| <= 0.99 eta / 0.01 = 0.1485) and above it, tilted to |cos| ~ 0.9995, with the room's side walls
  shading points whose shadow rays meet the light at |cos| in [0.25, 0.3].  Scene B adds a far triangle:
  the scene's extent breaks the error bound, so no mask may be set.
* The zero-direct-term skip: no shadow ray where the unoccluded direct term is exactly 0 (the light
  behind the surface).  Scene C puts the light under the floor, so most vertices have a zero term.

Each image is compared bitwise (float4 accumulation and RGBA8) with the CPU restatement."""
import numpy as np
import pytest

import _oracle as O
from _rt import rt

ETA = 0.15   # 0.0015 world units in the raw (x 100) coordinates the meshes are written in


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def quad(x0, x1, y0, y1, z0, z1):
    """Two triangles over x in [x0, x1] (y rising linearly from y0 to y1 along x), z in [z0, z1]; each
    triangle's first vertex is a right-angle corner (no sliver corner at the first vertex)."""
    v1, v2, v3, v4 = (x0, y0, z0), (x1, y1, z0), (x1, y1, z1), (x0, y0, z1)
    return np.array([v1 + v2 + v3, v3 + v4 + v1], np.float32)


def wall_x(x, z0, z1, y0, y1):
    v1, v2, v3, v4 = (x, y0, z0), (x, y1, z0), (x, y1, z1), (x, y0, z1)
    return np.array([v1 + v2 + v3, v3 + v4 + v1], np.float32)


def wall_z(z, x0, x1, y0, y1):
    v1, v2, v3, v4 = (x0, y0, z), (x1, y0, z), (x1, y1, z), (x0, y1, z)
    return np.array([v1 + v2 + v3, v3 + v4 + v1], np.float32)


WHITE, RED, GREEN = (0.7, 0.7, 0.7), (0.63, 0.065, 0.05), (0.1, 0.5, 0.1)
NOEM = (0.0, 0.0, 0.0)
LIGHT_EM = (47.8, 38.6, 31.1)
LY = 548.7   # the Cornell light's plane (MC/cornellbox/light.obj)


def scene_a(far=False):
    light = quad(213.0, 343.0, LY, LY, 227.0, 332.0)
    near = []
    # below the light (between a shaded point and the light): centre offsets 0.5, 0.9, 0.99 eta; the first
    # two tilted so their far edge reaches 0.95 / 0.99 eta (|cos| of the 4-unit-wide quad ~0.9995)
    near.append(quad(230.0, 234.0, LY - 0.05 * ETA, LY - 0.95 * ETA, 240.0, 320.0))
    near.append(quad(270.0, 274.0, LY - 0.81 * ETA, LY - 0.99 * ETA, 240.0, 320.0))
    near.append(quad(310.0, 314.0, LY - 0.99 * ETA, LY - 0.99 * ETA, 240.0, 320.0))
    # above it (beyond the light point for rays from below)
    near.append(quad(250.0, 254.0, LY + 0.05 * ETA, LY + 0.95 * ETA, 240.0, 320.0))
    near.append(quad(290.0, 294.0, LY + 0.81 * ETA, LY + 0.99 * ETA, 240.0, 320.0))
    near.append(quad(330.0, 334.0, LY + 0.99 * ETA, LY + 0.99 * ETA, 240.0, 320.0))
    floor = quad(0.0, 556.0, 0.0, 0.0, 0.0, 559.2)
    back = wall_z(559.2, 0.0, 556.0, 0.0, 548.8)
    left = wall_x(556.0, 0.0, 559.2, 0.0, 548.8)
    right = wall_x(0.0, 0.0, 559.2, 0.0, 548.8)
    block = quad(130.0, 290.0, 165.0, 165.0, 65.0, 225.0)   # a block top, for shadows on the floor
    meshes = [("floor", np.concatenate([floor, back]), WHITE, NOEM), ("left", left, RED, NOEM), ("right", right, GREEN, NOEM),
              ("block", block, WHITE, NOEM), ("near", np.concatenate(near), WHITE, NOEM), ("light", light, (0.65, 0.65, 0.65), LIGHT_EM)]
    if far:   # a triangle 50 world units away: 0.006 + 6e-5 x extent > 0.008, the bound fails
        meshes.insert(0, ("far", np.array([[5000.0, 0.0, 5000.0, 5010.0, 0.0, 5000.0, 5000.0, 10.0, 5000.0]], np.float32), WHITE, NOEM))
    return meshes


def scene_c():
    """The Cornell box (without its ceiling's light) lit from under the floor: the floor and the blocks'
    tops face away from the light, their direct terms are exactly 0."""
    out = []
    for (name, raw, alb, em) in O.cornell_meshes():
        raw = raw.copy()
        if name == "light":
            raw[:, 1::3] = -60.0
        out.append((name, raw, alb, em))
    return out


def build_rt(meshes):
    s = rt.Scene()
    for (_, raw, alb, em) in meshes:
        s.add_mesh(raw, alb, em)
    return s.build()


def test_scene_a_masks_the_adversarial_quads():
    sc = build_rt(scene_a())
    info = sc.info()
    assert info.n_tris <= 32 and info.n_leaf_boxes > 0
    # each light triangle's mask: both light triangles and the 12 near-coplanar quad triangles
    assert info.n_light_skip == 2 * 14, info.n_light_skip


def test_scene_b_bound_fails_no_mask():
    sc = build_rt(scene_a(far=True))
    assert sc.info().n_light_skip == 0


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["a", "b", "c"])
def test_adversarial_scene_matches_oracle(kind):
    meshes = scene_a() if kind == "a" else scene_a(far=True) if kind == "b" else scene_c()
    W, H, spp, seed = 128, 96, 16, 5
    c = rt.Context(0)
    try:
        c.upload(build_rt(meshes))
        c.resize(W, H)
        cam, _, _ = rt.camera_default(W, H)
        rgba, acc = c.render(cam, spp, seed=seed)
        assert c.stats().kernel == 1   # the leaf-box vertex kernel (the shortcuts live there)
    finally:
        c.close()
    oacc, orgba, _ = O.Scene(meshes).render(W, H, spp, seed=seed)
    same = np.mean(np.all(bits(acc) == bits(oacc), axis=-1))
    assert np.array_equal(bits(acc), bits(oacc)), f"{same:.4%} of pixels bitwise equal"
    assert np.array_equal(rgba, orgba)
