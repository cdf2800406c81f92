"""Host-side product code of librt_hip.so, on the CPU (no GPU needed):
scene packing vs the oracle, and the culling bounds of the prep kernel
(same __host__ __device__ code) proven conservative against the oracle's
per-pixel tests (MainState.cpp:257-327)."""
import ctypes

import numpy as np
import pytest

RAY_DIR = np.array([0.0, 0.0, -1.0, -1.0], np.float32)


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("scene_id", [1, 2, 3])
def test_reference_scenes_match_oracle(pkg, oracle, scene_id):
    got = pkg.Scene.reference(scene_id, 1)
    want = oracle.scene_reference(scene_id, 1)
    for k in ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
              "cube_colours"):
        assert np.array_equal(_bits(getattr(got, k)), _bits(getattr(want, k))), k


@pytest.mark.parametrize("args", [(512, 512, 4, 1, 1, 0.8), (1920, 1080, 16, 4, 2, 3.0),
                                  (4096, 4096, 256, 64, 3, 6.4), (97, 31, 0, 5, 9, 1.0)])
def test_synthetic_scene_matches_oracle(pkg, oracle, args):
    w, h, n, m, seed, k = args
    got = pkg.Scene.synthetic(w, h, n, m, seed=seed, k=k)
    want = oracle.scene_synthetic(w, h, n, m, seed, k)
    for key in ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
                "cube_colours"):
        assert np.array_equal(_bits(getattr(got, key)), _bits(getattr(want, key))), key


def test_cube_ops_match_oracle(pkg, oracle):
    rng = np.random.default_rng(3)
    for _ in range(200):
        ops = []
        for _ in range(int(rng.integers(1, 6))):
            kind = ["scale", "rotate", "translate"][int(rng.integers(0, 3))]
            lo, hi = {"scale": (0.01, 80), "rotate": (-7, 7), "translate": (-700, 700)}[kind]
            ops.append((kind, *rng.uniform(lo, hi, 3)))
        assert np.array_equal(_bits(pkg.cube_packed(ops)), _bits(oracle.cube(ops)))


def test_primary_ray_dir_and_angles(pkg, oracle):
    assert np.array_equal(pkg.primary_ray_dir(), RAY_DIR)
    for d in (0.0, 30.0, 80.0, 160.0, 210.0, 250.0, 359.0):
        assert np.float32(pkg.deg_to_rad(d)) == np.float32(oracle.deg2rad(d))


def test_pack_rgba8_matches_oracle(pkg, oracle):
    rng = np.random.default_rng(1)
    frame = rng.integers(-300, 600, (37, 53, 4)).astype(np.int32)
    assert np.array_equal(pkg.pack_rgba8(frame), oracle.pack_rgba8(frame))
    # (uint8) wrap of r, g, b; alpha forced opaque (MainState.cpp:1026-1036)
    px = pkg.pack_rgba8(np.array([[[257, -1, 255, 7]]], np.int32))[0, 0]
    assert px == (1 | (255 << 8) | (255 << 16) | (255 << 24))


# ---------------------------------------------------------------------------
# culling bounds
# ---------------------------------------------------------------------------
def tile_shape(pkg):
    w, h = ctypes.c_int32(), ctypes.c_int32()
    assert pkg.library().rt_debug_tile_shape(ctypes.byref(w), ctypes.byref(h)) == 0
    return w.value, h.value


def block_shape(pkg):
    w, h = ctypes.c_int32(), ctypes.c_int32()
    assert pkg.library().rt_debug_block_shape(ctypes.byref(w), ctypes.byref(h)) == 0
    return w.value, h.value


def classified_shapes(pkg):
    """The rectangles the coarse kernel classifies: row blocks (and whole
    tiles, which the tests keep checking as a stronger property)."""
    tw, th = tile_shape(pkg)
    bw, bh = block_shape(pkg)
    assert bw == tw and th % bh == 0
    return sorted({(tw, th), (bw, bh)})


def classify_tile(cls, is_tri, x0, y0, tw, th):
    """numpy float32 mirror of the trace kernel's classify() (rt_device.hip)
    on a tw x th wave tile."""
    f = np.float32
    kw, kh = f(tw - 1), f(th - 1)
    a = cls[:4].astype(np.float32)
    b = cls[4:].astype(np.float32)
    x0, y0 = f(x0), f(y0)
    if is_tri:
        xl, xh = x0 - a[0], (x0 + kw) - a[0]
        yl, yh = y0 - a[1], (y0 + kh) - a[1]
        u1, u2, u3, u4 = a[2] * xl, a[2] * xh, a[3] * yl, a[3] * yh
        v1, v2, v3, v4 = b[0] * xl, b[0] * xh, b[1] * yl, b[1] * yh
        umin, umax = min(u1, u2) + min(u3, u4), max(u1, u2) + max(u3, u4)
        vmin, vmax = min(v1, v2) + min(v3, v4), max(v1, v2) + max(v3, v4)
        g = b[2]
        out = (umax < -g or umin > f(1) + g or vmax < -g or vmin > f(1) + g
               or umin + vmin > f(1) + g)
        inside = (umin > g and umax < f(1) - g and vmin > g and vmax < f(1) - g
                  and umax + vmax < f(1) - g)
        return not out, bool(inside)
    dx = max(max(x0 - a[0], a[0] - (x0 + kw)), f(0))
    dy = max(max(y0 - a[1], a[1] - (y0 + kh)), f(0))
    return not (dx * dx + dy * dy > a[2]), False


def random_triangles(rng, w, h, n):
    tris = []
    for i in range(n):
        kind = i % 5
        c = rng.uniform([-20, -20, -120], [w + 20, h + 20, 20])
        if kind == 0:    # ordinary
            v = c + rng.uniform(-60, 60, (3, 3))
        elif kind == 1:  # sliver: nearly collinear in xy
            d = rng.uniform(-80, 80, 3)
            v = np.stack([c, c + d, c + d * rng.uniform(0.2, 0.8) + rng.uniform(-1e-3, 1e-3, 3)])
        elif kind == 2:  # tiny
            v = c + rng.uniform(-0.05, 0.05, (3, 3))
        elif kind == 3:  # huge, mostly off-frame
            v = c + rng.uniform(-3000, 3000, (3, 3))
        else:            # axis-aligned edges through pixel centres
            x, y = np.floor(c[:2])
            s = float(rng.integers(1, 40))
            v = np.array([[x, y, c[2]], [x + s, y, c[2] - 3], [x, y + s, c[2] + 2]])
        tris.append(v.astype(np.float32))
    return tris


def classify_pixels(cls, xs, ys):
    """numpy float32 mirror of test_primitive's per-pixel pre-classification
    (partial tiles): returns (out, inside) masks."""
    f = np.float32
    a = cls[:4].astype(np.float32)
    b = cls[4:].astype(np.float32)
    xl = xs.astype(np.float32) - a[0]
    ux, vx = a[2] * xl, b[0] * xl
    yl = ys.astype(np.float32) - a[1]
    ul = ux + a[3] * yl
    vl = vx + b[1] * yl
    wl = ul + vl
    g = b[2]
    out = (ul < -g) | (ul > f(1) + g) | (vl < -g) | (vl > f(1) + g) | (wl > f(1) + g)
    inside = (ul > g) & (ul < f(1) - g) & (vl > g) & (vl < f(1) - g) & (wl < f(1) - g)
    return out, inside


def wide_tile_shape(pkg):
    w, h = ctypes.c_int32(), ctypes.c_int32()
    assert pkg.library().rt_debug_tile_shape_wide(ctypes.byref(w), ctypes.byref(h)) == 0
    return w.value, h.value


@pytest.mark.parametrize("build", ["narrow", "wide"])
@pytest.mark.parametrize("band", [(0, 160), (37, 121)])
def test_triangle_box_and_tile_classifier_are_conservative(pkg, oracle, band, build):
    """Both wave-tile builds (16x16 and 128x2 tiles; each has its own
    classifier margin for its tile span)."""
    w, h = 176, 160
    rb, re = band
    if build == "narrow":
        tw, th = tile_shape(pkg)
        shapes = classified_shapes(pkg)
        prep = pkg.debug_triangle_prep
    else:
        tw, th = wide_tile_shape(pkg)
        assert (tw, th) == (128, 2)
        shapes = [(tw, th)]
        prep = pkg.debug_triangle_prep_wide
    rng = np.random.default_rng(7 + rb)
    n_inside_tiles = n_skip_tiles = 0
    for v in random_triangles(rng, w, h, 150):
        ok, box, cls = prep(v[0], v[1], v[2], RAY_DIR, w, rb, re)
        hits = oracle.tri_grid(v[0], v[1], v[2], RAY_DIR, 0, rb, w, re - rb)
        if not ok:
            assert not hits.any()
            continue
        ys, xs = np.nonzero(hits)
        if len(xs):
            assert box[0] <= xs.min() and xs.max() <= box[2]
            assert box[1] <= ys.min() + rb and ys.max() + rb <= box[3]
        # per-pixel pre-classification of every pixel inside the padded box
        x0, x1 = max(box[0] - tw, 0), min(box[2] + tw, w - 1)
        y0, y1 = max(box[1] - th, rb), min(box[3] + th, re - 1)
        if x0 <= x1 and y0 <= y1:
            ys, xs = np.mgrid[y0:y1 + 1, x0:x1 + 1]
            out_px, in_px = classify_pixels(cls, xs, ys)
            sub = hits[y0 - rb:y1 - rb + 1, x0:x1 + 1].astype(bool)
            assert not (out_px & sub).any(), v
            assert not (in_px & ~sub).any(), v
        for sw, sh in shapes:
            for ty in range(rb, re, sh):
                for tx in range(0, w, sw):
                    if box[0] > tx + sw - 1 or box[2] < tx or box[1] > ty + sh - 1 or box[3] < ty:
                        continue  # the kernel classifies only rectangles the box touches
                    keep, inside = classify_tile(cls, True, tx, ty, sw, sh)
                    tile = hits[ty - rb:ty - rb + sh, tx:tx + sw]
                    if not keep:
                        n_skip_tiles += 1
                        assert not tile.any(), (v, tx, ty, sw, sh)
                    if inside:
                        n_inside_tiles += 1
                        assert tile.all(), (v, tx, ty, sw, sh)
    assert n_inside_tiles > 0 and n_skip_tiles > 0  # the classifier does something


@pytest.mark.parametrize("tile", [(16, 16), (64, 4), (128, 2)])
def test_triangle_t_bounds_hold(pkg, oracle, tile):
    """The coarse depth cull's triangle bounds (tri_t_bounds): for every
    hitting pixel of a tile, the reference's fp64 t lies in [lo, hi], so its
    float closest value lies in [(float)lo, (float)hi] -- the property the
    cull's strict comparisons rely on.  Random, sliver, tiny, huge and
    axis-aligned triangles; tiles of both wave-tile shapes around them."""
    w, h = 176, 160
    tw, th = tile
    rng = np.random.default_rng(29 + tw)
    n_checked = 0
    for v in random_triangles(rng, w, h, 150):
        ok, box, _ = pkg.debug_triangle_prep(v[0], v[1], v[2], RAY_DIR, w, 0, h)
        if not ok or box[0] > box[2]:
            continue
        for _ in range(6):
            tx = int(rng.integers(max(box[0] - tw, 0), box[2] + 1)) // tw * tw
            ty = int(rng.integers(max(box[1] - th, 0), box[3] + 1)) // th * th
            b = pkg.debug_triangle_t_bounds(v[0], v[1], v[2], RAY_DIR, w, 0, h,
                                            tx, tx + tw - 1, ty, ty + th - 1)
            if b is None:
                continue
            ts = oracle.tri_t_grid(v[0], v[1], v[2], RAY_DIR, tx, ty, tw, th)
            hit = ~np.isnan(ts)
            if not hit.any():
                continue
            lo, hi = b
            assert (ts[hit] >= lo).all() and (ts[hit] <= hi).all(), (v, tx, ty, lo, hi)
            f = ts[hit].astype(np.float32)
            assert (f >= np.float32(lo)).all() and (f <= np.float32(hi)).all()
            n_checked += int(hit.sum())
    assert n_checked > 10000


@pytest.mark.parametrize("tile", [(16, 16), (64, 4), (128, 2)])
def test_triangle_t_bounds_hold_far_from_origin(pkg, oracle, tile):
    """The same bounds where their error margin is largest: the margin grows
    with the pixel coordinates (M0 + Mx |x| + My |y|), and configs 4 and 5
    put tiles at x, y up to 16383.  Triangles of every kind are moved to
    4000-16200 px from the origin on a 16384 x 16384 frame."""
    w = h = 16384
    tw, th = tile
    rng = np.random.default_rng(71 + tw)
    n_checked = 0
    for v in random_triangles(rng, 176, 160, 150):
        off = np.float32([rng.uniform(4000, 16000), rng.uniform(4000, 16000), 0.0])
        v = (v + off).astype(np.float32)
        ok, box, _ = pkg.debug_triangle_prep(v[0], v[1], v[2], RAY_DIR, w, 0, h)
        if not ok or box[0] > box[2]:
            continue
        for _ in range(6):
            tx = int(rng.integers(max(box[0] - tw, 0), box[2] + 1)) // tw * tw
            ty = int(rng.integers(max(box[1] - th, 0), box[3] + 1)) // th * th
            b = pkg.debug_triangle_t_bounds(v[0], v[1], v[2], RAY_DIR, w, 0, h,
                                            tx, tx + tw - 1, ty, ty + th - 1)
            if b is None:
                continue
            ts = oracle.tri_t_grid(v[0], v[1], v[2], RAY_DIR, tx, ty, tw, th)
            hit = ~np.isnan(ts)
            if not hit.any():
                continue
            lo, hi = b
            assert (ts[hit] >= lo).all() and (ts[hit] <= hi).all(), (v, tx, ty, lo, hi)
            f = ts[hit].astype(np.float32)
            assert (f >= np.float32(lo)).all() and (f <= np.float32(hi)).all()
            n_checked += int(hit.sum())
    assert n_checked > 10000


def test_sphere_box_and_tile_classifier_are_conservative(pkg, oracle):
    w, h = 160, 128
    shapes = classified_shapes(pkg)
    rng = np.random.default_rng(11)
    for i in range(120):
        c = np.float32([rng.uniform(-30, w + 30), rng.uniform(-30, h + 30),
                        rng.uniform(-150, 10), [1.0, 0.5, 3.0][i % 3]])
        r = np.float32([0.0, 1e-3, 0.7, 5.0, 25.0, 90.0][i % 6] * rng.uniform(0.5, 1.5))
        ok, box, cls = pkg.debug_sphere_prep(c, r, RAY_DIR, w, 0, h)
        assert ok
        hits = oracle.sphere_grid(c, r, RAY_DIR, 0, 0, w, h)
        ys, xs = np.nonzero(hits)
        if len(xs):
            assert box[0] <= xs.min() and xs.max() <= box[2]
            assert box[1] <= ys.min() and ys.max() <= box[3]
        elif box[0] > box[2]:
            continue
        for tw, th in shapes:
            for ty in range(0, h, th):
                for tx in range(0, w, tw):
                    keep, _ = classify_tile(cls, False, tx, ty, tw, th)
                    if not keep:
                        assert not hits[ty:ty + th, tx:tx + tw].any(), (c, r, tx, ty, tw, th)


def _decode_png(path):
    """Minimal decoder for the encoder's own output (8-bit RGBA, filter 0)."""
    import struct
    import zlib
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        kind, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(kind + body) & 0xFFFFFFFF
        if kind == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", body[:10])
            assert (depth, ctype) == (8, 6)
        elif kind == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 4 * w)
    assert not raw[:, 0].any()
    return raw[:, 1:].reshape(h, w, 4)


def test_encode_png_round_trip(pkg, oracle, tmp_path):
    """MainState::encodePNG (MainState.cpp:410-417): the Texture's RGBA8
    bytes survive the PNG round trip."""
    frame = oracle.trace(oracle.scene_reference(1), 64, 48)
    rgba = pkg.pack_rgba8(frame)
    path = tmp_path / "ray.png"
    pkg.encode_png(str(path), rgba)
    got = _decode_png(str(path))
    assert np.array_equal(got, rgba.astype("<u4").view(np.uint8).reshape(48, 64, 4))
    assert (got[..., 3] == 255).all()
