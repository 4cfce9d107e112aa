"""Screen-tile sharding of a frame across GPUs (one process per GPU).

Mirrors ``buildUnits`` in csrc/mrt_renderer.hip: the reference's 16x16 tiling
(Renderer.cpp:33-38, 117-135) cut into 8-row bands ("units"); unit (tile t, band b) belongs
to rank (t + b) % world.  Pixel slots of a rank are its units' pixels in order, column-major inside a unit.
The renderer writes a rank's frame as a packed int32 array in slot order; rank 0 gathers the
packed arrays (one RCCL gather of pixelSlotsMax int32 per rank) and scatters them into the
bitmap.  Every pixel has exactly one owner, so no reduction is needed and the assembled frame
is bit-identical to a single-GPU render (sample streams are per-pixel pure functions).
"""
import math

import numpy as np

NUMBER_OF_TILES = 256  # Constants.hpp:50


def units(width, height):
    side = int(math.sqrt(NUMBER_OF_TILES))
    bx, by = width // side, height // side
    if bx <= 0 or by <= 0:
        raise ValueError("width and height must be >= 16")
    domain = (width // bx) * (height // by)
    res = width * height
    blocks = []
    for j in range(NUMBER_OF_TILES):
        tile = np.float32(j) / np.float32(NUMBER_OF_TILES)
        rb = int(math.floor(float(np.float32(tile * np.float32(domain))) + 0.5))  # roundf, x >= 0
        if rb not in blocks:
            blocks.append(rb)
    out = []
    for t, rb in enumerate(blocks):
        pixel = rb * bx % res
        start_y = ((pixel // width) * by) % height
        start_x = pixel % width
        b = 0
        while b * 8 < by:
            h = min(8, by - 8 * b)
            y0 = start_y + 8 * b
            while h > 0 and (y0 + h - 1) * width + start_x + bx - 1 >= res:
                h -= 1
            if h > 0:
                out.append((start_x, y0, bx, h, t + b))
            b += 1
    return out


def rank_units(width, height, rank, world):
    """Unit (tile t, band b) belongs to rank (t + b) % world, which spreads the short last
    band of every tile over the ranks."""
    return [u[:4] for u in units(width, height) if u[4] % world == rank]


def slot_pixels(width, height, rank, world):
    """Bitmap index of every pixel slot of `rank`, in slot order."""
    idx = []
    for (x0, y0, w, h) in rank_units(width, height, rank, world):
        xs = x0 + np.repeat(np.arange(w), h)
        ys = y0 + np.tile(np.arange(h), w)
        idx.append(ys * width + xs)
    return np.concatenate(idx) if idx else np.zeros(0, np.int64)


def max_slots(width, height, world):
    return max(len(slot_pixels(width, height, r, world)) for r in range(world))


def pack(bitmap, width, height, rank, world, slots_max=None):
    """The packed buffer a rank produces (numpy restatement of k_accumulate's packed output)."""
    idx = slot_pixels(width, height, rank, world)
    n = slots_max if slots_max is not None else len(idx)
    out = np.zeros(n, np.int32)
    out[: len(idx)] = bitmap[idx]
    return out


def unpack(gathered, width, height, world, bitmap):
    """Rank-0 frame assembly (numpy restatement of k_unpack)."""
    for r in range(world):
        idx = slot_pixels(width, height, r, world)
        bitmap[idx] = gathered[r, : len(idx)]
    return bitmap
