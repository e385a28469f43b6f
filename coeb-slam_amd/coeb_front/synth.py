"""Synthetic TUM-like input for parity tests and the benchmark.

No dataset ships with the reference and there is no network, so every frame is generated:
a torus-wrapped canvas of 40-80 axis-aligned rectangles (uniform intensity, half with 3-px
soft ramps), translated by (dx, dy) = (+2, +1) px per frame, plus fresh uniform noise in
[-6, 6].  A constant depth Z = 2.0 m makes the image motion exactly the camera translation
t = (dx*Z/fx, dy*Z/fy, 0), which is what the matcher's motion model is given.
"""
import numpy as np

# Examples/RGB-D/tum_bag.yaml
TUM_FX, TUM_FY, TUM_CX, TUM_CY, TUM_BF = 535.4, 539.2, 320.1, 247.6, 40.0
SHIFT = (2, 1)
DEPTH_Z = 2.0


def make_canvas(w, h, seed):
    rng = np.random.default_rng(seed)
    canvas = np.full((h, w), rng.integers(40, 200), dtype=np.float64)
    nrect = int(rng.integers(40, 81))
    for r in range(nrect):
        rw = int(rng.integers(16, max(17, w // 4)))
        rh = int(rng.integers(16, max(17, h // 4)))
        x0 = int(rng.integers(0, w))
        y0 = int(rng.integers(0, h))
        val = float(rng.integers(0, 256))
        ys = (y0 + np.arange(rh)) % h
        xs = (x0 + np.arange(rw)) % w
        if r % 2 == 0:
            canvas[np.ix_(ys, xs)] = val
        else:
            dy = np.minimum(np.arange(rh), np.arange(rh)[::-1])
            dx = np.minimum(np.arange(rw), np.arange(rw)[::-1])
            d = np.minimum(dy[:, None], dx[None, :])
            alpha = np.minimum(1.0, (d + 1) / 4.0)
            old = canvas[np.ix_(ys, xs)]
            canvas[np.ix_(ys, xs)] = np.rint(alpha * val + (1 - alpha) * old)
    return canvas.astype(np.int16)


def frame_from_canvas(canvas, k, noise_seed):
    h, w = canvas.shape
    img = np.roll(canvas, (k * SHIFT[1], k * SHIFT[0]), axis=(0, 1))
    noise = np.random.default_rng(noise_seed).integers(-6, 7, size=(h, w), dtype=np.int16)
    return np.clip(img + noise, 0, 255).astype(np.uint8)


def make_frames(w, h, n, seed=1000, first=0):
    """n consecutive frames (uint8, n x h x w) of one sequence."""
    canvas = make_canvas(w, h, seed)
    out = np.empty((n, h, w), dtype=np.uint8)
    for i in range(n):
        k = first + i
        out[i] = frame_from_canvas(canvas, k, seed * 7919 + k + 1)
    return out


def make_depth(w, h, z=DEPTH_Z):
    return np.full((h, w), z, dtype=np.float32)


def motion_pose(z=DEPTH_Z, fx=TUM_FX, fy=TUM_FY):
    """Tcw of frame k+1 relative to Tcw(k) = I for the synthetic (+2,+1) px motion."""
    T = np.eye(4, dtype=np.float32)
    T[0, 3] = np.float32(SHIFT[0] * z / fx)
    T[1, 3] = np.float32(SHIFT[1] * z / fy)
    return T


def dynamic_inputs(w, h, seed=7, area_flag=False):
    """Boxes + T_M + blur_flag of config 3.  area_flag=True forces the
    'dynamic area > 200000' branch with three large boxes."""
    sx, sy = w / 640.0, h / 480.0
    if not area_flag:
        boxes = np.array([[200, 100, 320, 400], [400, 150, 480, 380]], dtype=np.float32)
    else:
        boxes = np.array([[20, 20, 330, 460], [330, 40, 620, 470], [100, 300, 600, 470]],
                         dtype=np.float32)
    boxes[:, [0, 2]] *= sx
    boxes[:, [1, 3]] *= sy
    rng = np.random.default_rng(seed)
    pts = []
    for i in range(30):
        b = boxes[i % len(boxes)]
        pts.append([rng.uniform(b[0], b[2]), rng.uniform(b[1], b[3])])
    for i in range(30):
        pts.append([rng.uniform(0, w - 1), rng.uniform(0, h - 1)])
    tm = np.array(pts, dtype=np.float32)
    blur = np.array([0, 1, 1][:len(boxes)], dtype=np.int32)
    return boxes, tm, blur


def make_local_map(xw, desc, octave, Tcw, w, h, fx=TUM_FX, fy=TUM_FY, cx=TUM_CX, cy=TUM_CY, bf=TUM_BF,
                   nlevels=8, seed=0, dup_frac=0.3, n_distract=300, jitter=1.0):
    """A synthetic vpLocalMapPoints snapshot after Frame::isInFrustum (Frame.cc:445-501) for the
    local-map projection search: the map points xw [n,3] projected with Tcw (+ Gaussian jitter
    in px), predicted level = octave +- 1, view cosines on both sides of 0.998
    (RadiusByViewingCos), plus near-duplicates (a few descriptor bits flipped: ratio-test and
    claim conflicts) and random distractors, shuffled.  Returns a dict of the coeb_localmap
    arrays (in_view, proj_x, proj_y, proj_xr, level, view_cos, descriptor, observations)."""
    rng = np.random.default_rng(seed)
    xw = np.asarray(xw, np.float32).reshape(-1, 3)
    desc = np.asarray(desc, np.uint8).reshape(-1, 32)
    octave = np.asarray(octave, np.int32)
    R, t = np.asarray(Tcw, np.float32)[:3, :3], np.asarray(Tcw, np.float32)[:3, 3]
    pc = xw @ R.T + t
    z = pc[:, 2]
    ok = z > 0
    invz = np.where(ok, 1.0 / np.where(ok, z, 1), 0).astype(np.float32)
    u = (fx * pc[:, 0] * invz + cx).astype(np.float32)
    v = (fy * pc[:, 1] * invz + cy).astype(np.float32)
    n = len(xw)
    lvl = np.clip(octave + rng.integers(-1, 2, n), 0, nlevels - 1).astype(np.int32)
    pts = [dict(u=u, v=v, ur=(u - bf * invz).astype(np.float32), lvl=lvl, desc=desc, ok=ok)]
    nd = int(n * dup_frac)
    if nd:
        pick = rng.choice(n, nd, replace=True)
        d = desc[pick].copy()
        for k in range(nd):                 # flip 0..12 random bits
            for b in rng.integers(0, 256, rng.integers(0, 13)):
                d[k, b >> 3] ^= np.uint8(1 << (b & 7))
        pts.append(dict(u=u[pick] + rng.normal(0, 2, nd).astype(np.float32),
                        v=v[pick] + rng.normal(0, 2, nd).astype(np.float32),
                        ur=(u[pick] - bf * invz[pick]).astype(np.float32), lvl=lvl[pick], desc=d, ok=ok[pick]))
    if n_distract:
        pts.append(dict(u=rng.uniform(-20, w + 20, n_distract).astype(np.float32),
                        v=rng.uniform(-20, h + 20, n_distract).astype(np.float32),
                        ur=rng.uniform(-50, w, n_distract).astype(np.float32),
                        lvl=rng.integers(0, nlevels, n_distract).astype(np.int32),
                        desc=rng.integers(0, 256, (n_distract, 32)).astype(np.uint8),
                        ok=np.ones(n_distract, bool)))
    cat = {k: np.concatenate([p[k] for p in pts]) for k in pts[0]}
    m = len(cat["u"])
    order = rng.permutation(m)
    ju = rng.normal(0, jitter, m).astype(np.float32)
    jv = rng.normal(0, jitter, m).astype(np.float32)
    px = (cat["u"] + ju)[order].astype(np.float32)
    py = (cat["v"] + jv)[order].astype(np.float32)
    in_view = (cat["ok"][order] & (px >= 0) & (px < w) & (py >= 0) & (py < h)).astype(np.uint8)
    cos = np.where(rng.random(m) < 0.5, rng.uniform(0.9981, 1.0, m), rng.uniform(0.5, 0.998, m)).astype(np.float32)
    return dict(in_view=in_view, proj_x=px, proj_y=py, proj_xr=(cat["ur"] + ju)[order].astype(np.float32),
                level=np.where(in_view > 0, cat["lvl"][order], -1).astype(np.int32), view_cos=cos,
                descriptor=np.ascontiguousarray(cat["desc"][order]),
                observations=rng.choice(np.array([0, 1, 2, 3], np.int32), m, p=[0.3, 0.2, 0.3, 0.2]).astype(np.int32))


def make_keyframe_points(xw, desc, octave, angle, scale_factor=1.2, nlevels=8, seed=0, n_distract=200,
                         invalid_frac=0.1, far_frac=0.05):
    """A synthetic pKF->GetMapPointMatches() snapshot for the relocalisation search: the map
    points xw [n,3] of a KeyFrame at Twc = I, with mfMaxDistance = |x| * scale[octave] and
    mfMinDistance = mfMaxDistance / scale[nlevels-1] (MapPoint::UpdateNormalAndDepth,
    MapPoint.cc:352-369) jittered by +-10 % (a few pushed out of the invariance range), a
    fraction invalid (NULL / bad), plus random distractors.  Returns a dict of the
    coeb_keyframe_points arrays (valid, world_pos, descriptor, max_distance, min_distance, angle)."""
    rng = np.random.default_rng(seed)
    xw = np.asarray(xw, np.float32).reshape(-1, 3)
    n = len(xw)
    sc = np.float32(scale_factor) ** np.arange(nlevels, dtype=np.float32)
    dist = np.sqrt((xw.astype(np.float64) ** 2).sum(1)).astype(np.float32)
    maxd = (dist * sc[np.clip(octave, 0, nlevels - 1)] * rng.uniform(0.9, 1.1, n)).astype(np.float32)
    far = rng.random(n) < far_frac
    maxd[far] *= np.float32(0.3)                     # outside [0.8 min, 1.2 max]
    mind = (maxd / sc[-1]).astype(np.float32)
    dx = rng.uniform(-1.5, 1.5, (n_distract, 3)).astype(np.float32)
    dx[:, 2] = rng.uniform(1.0, 4.0, n_distract)
    dd = np.sqrt((dx.astype(np.float64) ** 2).sum(1)).astype(np.float32)
    dmax = (dd * sc[rng.integers(0, nlevels, n_distract)]).astype(np.float32)
    return dict(valid=np.concatenate([(rng.random(n) >= invalid_frac), np.ones(n_distract, bool)]).astype(np.uint8),
                world_pos=np.ascontiguousarray(np.concatenate([xw, dx]), np.float32),
                descriptor=np.ascontiguousarray(np.concatenate([np.asarray(desc, np.uint8).reshape(-1, 32),
                                                                rng.integers(0, 256, (n_distract, 32)).astype(np.uint8)])),
                max_distance=np.concatenate([maxd, dmax]).astype(np.float32),
                min_distance=np.concatenate([mind, (dmax / sc[-1])]).astype(np.float32),
                angle=np.concatenate([np.asarray(angle, np.float32),
                                      rng.uniform(0, 360, n_distract).astype(np.float32)]).astype(np.float32))


def rotated_pose(deg, axis=1, t=(0.02, -0.01, 0.03)):
    """Tcw with a rotation of `deg` degrees about one axis plus a translation (relocalisation
    poses that are not pure translations)."""
    a = np.deg2rad(deg)
    c, s = np.cos(a), np.sin(a)
    R = np.eye(3)
    i, j = [(1, 2), (0, 2), (0, 1)][axis]
    R[i, i] = c; R[j, j] = c; R[i, j] = -s; R[j, i] = s
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = R.astype(np.float32)
    T[:3, 3] = np.asarray(t, np.float32)
    return T


def make_pose_problem(n=600, seed=0, outlier_frac=0.2, mono_frac=0.3, noise=0.7, nlevels=8, scale_factor=1.2,
                      w=640, h=480, fx=TUM_FX, fy=TUM_FY, cx=TUM_CX, cy=TUM_CY, bf=TUM_BF, init_err=(0.02, 0.03)):
    """A synthetic Optimizer::PoseOptimization input: n keypoints of which most hold a MapPoint
    seen from a true pose (rotation ~3 deg, translation ~0.1 m) with Gaussian pixel noise at
    their octave's scale, a fraction of gross outliers (wrong 3-D points), a fraction without
    depth (mvuRight = -1, monocular edges), and an initial pose perturbed by init_err
    (rad, m).  Returns dict(kps, has_mp, xw, ur, Tcw_init, Tcw_true)."""
    rng = np.random.default_rng(seed)

    def pose(rv, t):
        th = np.linalg.norm(rv)
        K = np.array([[0, -rv[2], rv[1]], [rv[2], 0, -rv[0]], [-rv[1], rv[0], 0]])
        R = np.eye(3) if th == 0 else np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K
        T = np.eye(4)
        T[:3, :3] = R
        T[:3, 3] = t
        return T

    Ttrue = pose(rng.normal(0, 0.03, 3), rng.normal(0, 0.1, 3))
    Tinit = pose(rng.normal(0, init_err[0], 3), rng.normal(0, init_err[1], 3)) @ Ttrue
    z = rng.uniform(1.0, 6.0, n)
    u = rng.uniform(20, w - 20, n)
    v = rng.uniform(20, h - 20, n)
    pc = np.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], 1)
    Rt, tt = Ttrue[:3, :3], Ttrue[:3, 3]
    xw = (pc - tt) @ Rt                                        # Xw = R^T (Xc - t)
    octave = rng.integers(0, nlevels, n).astype(np.int32)
    sig = np.float64(scale_factor) ** octave
    kps = np.zeros(n, np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                                ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")]))
    kps["x"] = u + rng.normal(0, noise, n) * sig
    kps["y"] = v + rng.normal(0, noise, n) * sig
    kps["octave"] = octave
    kps["class_id"] = -1
    ur = (kps["x"] - bf / z + rng.normal(0, noise, n) * sig).astype(np.float32)
    ur[rng.random(n) < mono_frac] = -1.0
    out = rng.random(n) < outlier_frac
    xw[out] += rng.normal(0, 0.5, (out.sum(), 3))
    has = (rng.random(n) < 0.9).astype(np.uint8)
    return dict(kps=kps, has_mp=has, xw=xw.astype(np.float32), ur=ur, Tcw_init=Tinit.astype(np.float32),
                Tcw_true=Ttrue.astype(np.float32), gross=out)


def _texture(rng, w, h, density=400):
    tex = np.full((h, w), int(rng.integers(60, 200)), np.int16)
    for _ in range(max(1, w * h // density)):
        s = int(rng.integers(4, 11))
        x0, y0 = int(rng.integers(0, w - s)), int(rng.integers(0, h - s))
        tex[y0:y0 + s, x0:x0 + s] = int(rng.integers(0, 256))
    return tex


def moving_object_pair(w, h, seed=0, n_small=600, obj=(200, 120, 160, 200), obj_shift=(-5, 4), noise=True):
    """A frame pair for Frame::ProcessMovingObject (Frame.cc:311-393).  A sideways camera
    translation gives every static point a flow parallel to SHIFT whose length depends on its
    depth: a far textured background (make_canvas plus n_small 4-12 px squares) moves by SHIFT,
    three nearer textured panels by 2x and 3x SHIFT, and an object rectangle obj = (x, y, w, h)
    moves by obj_shift, off the epipolar direction.  Returns (prev, cur, object box
    (xmin, ymin, xmax, ymax) in cur)."""
    frames, boxes = moving_object_sequence(w, h, 2, seed, n_small, obj, obj_shift, noise)
    return frames[0], frames[1], boxes[1]


def moving_object_sequence(w, h, n, seed=0, n_small=600, obj=(200, 120, 160, 200), obj_shift=(-5, 4), noise=True):
    """n frames of moving_object_pair's scene (frame k: background and panels k steps of the
    camera motion on, the object k steps of obj_shift); returns (frames (n, h, w) u8, object box
    (xmin, ymin, xmax, ymax) per frame as float32 (n, 4)).  The object must stay inside the
    frame: n * |obj_shift| is limited by obj's margins."""
    rng = np.random.default_rng(seed + 31337)
    canvas = make_canvas(w, h, seed).astype(np.int16)
    for _ in range(n_small):
        s = int(rng.integers(4, 13))
        x0, y0 = int(rng.integers(0, w - s)), int(rng.integers(0, h - s))
        canvas[y0:y0 + s, x0:x0 + s] = int(rng.integers(0, 256))
    layers = []
    for m, (px, py) in zip((2, 3, 2), ((40, 40), (420, 60), (380, 300))):
        pw, ph = int(rng.integers(120, 180)), int(rng.integers(100, 150))
        layers.append((_texture(rng, pw, ph), px, py, (m * SHIFT[0], m * SHIFT[1])))
    ox, oy, ow, oh = obj
    layers.append((_texture(rng, ow, oh), ox, oy, obj_shift))
    frames = np.empty((n, h, w), np.uint8)
    boxes = np.empty((n, 4), np.float32)
    for k in range(n):
        img = np.roll(canvas, (k * SHIFT[1], k * SHIFT[0]), axis=(0, 1)).copy()
        for tex, px, py, sh in layers:
            x, y = px + k * sh[0], py + k * sh[1]
            th, tw = tex.shape
            x0, y0, x1, y1 = max(x, 0), max(y, 0), min(x + tw, w), min(y + th, h)
            if x1 > x0 and y1 > y0:
                img[y0:y1, x0:x1] = tex[y0 - y:y1 - y, x0 - x:x1 - x]
        if noise:
            img = img + np.random.default_rng(seed * 7919 + k + 1).integers(-3, 4, size=(h, w), dtype=np.int16)
        frames[k] = np.clip(img, 0, 255).astype(np.uint8)
        x, y = ox + k * obj_shift[0], oy + k * obj_shift[1]
        boxes[k] = (x, y, x + ow, y + oh)
    return frames, boxes


def _bounce(t, lo, hi):
    """Triangle wave: position t folded into [lo, hi] (an object bouncing between two walls)."""
    span = hi - lo
    if span <= 0:
        return lo
    m = t % (2 * span)
    return lo + (m if m <= span else 2 * span - m)


def tracking_sequence(w, h, n, first=0, seed=1000, obj_size=(120, 160), obj_speed=(-5, 4)):
    """Frames first .. first+n-1 of an endless RGB-D tracking sequence (BASELINE configs[4]):
    make_frames' background (the camera motion of motion_pose at depth DEPTH_Z) with a textured
    object bouncing around the image at obj_speed px/frame, off the epipolar direction (the
    YOLO box is its bounding box).  Frame k depends on k only, so shards of the sequence agree
    with the whole.  Returns (gray (n, h, w) u8, boxes (n, 4) f32 xyxy)."""
    canvas = make_canvas(w, h, seed)
    rng = np.random.default_rng(seed + 4711)
    ow, oh = obj_size
    tex = _texture(rng, ow, oh, density=150)
    x0, y0 = w // 3, h // 4
    frames = np.empty((n, h, w), np.uint8)
    boxes = np.empty((n, 4), np.float32)
    for i in range(n):
        k = first + i
        img = np.roll(canvas, (k * SHIFT[1], k * SHIFT[0]), axis=(0, 1)).copy()
        x = _bounce(x0 + k * obj_speed[0], 8, w - ow - 8)
        y = _bounce(y0 + k * obj_speed[1], 8, h - oh - 8)
        img[y:y + oh, x:x + ow] = tex
        noise = np.random.default_rng(seed * 7919 + k + 1).integers(-6, 7, size=(h, w), dtype=np.int16)
        frames[i] = np.clip(img + noise, 0, 255).astype(np.uint8)
        boxes[i] = (x, y, x + ow, y + oh)
    return frames, boxes


def rgbd_from_gray(gray, z=DEPTH_Z, depth_factor=5000.0):
    """TUM-style raw input for GrabImageRGBD: 8UC3 RGB with R = G = B = gray (RGB2GRAY gives
    gray back exactly: the 14-bit weights sum to 2^14) and 16UC1 depth in 1/depth_factor m."""
    rgb = np.repeat(np.asarray(gray, np.uint8)[..., None], 3, axis=-1)
    d = np.full(gray.shape, int(round(z * depth_factor)), np.uint16)
    return np.ascontiguousarray(rgb), d
