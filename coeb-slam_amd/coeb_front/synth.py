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
