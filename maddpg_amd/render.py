"""Headless ``--display`` (``experiments/train.py:150-154``).

The reference calls MPE's ``env.render()`` (a pyglet window: every entity a
filled circle of its ``size`` and ``color``, shared camera spanning [-1, 1]
around the origin) after each policy step and trains nothing.  There is no
display on a GPU box, so the frames are rasterised here and written as PNG
files (stdlib zlib, no imaging package), plus one ``positions.npz`` with every
frame's entity positions.  Entity sizes follow the scenario tables of the
device env (``mdp_api.cpp`` make_env); colours are the upstream scenarios'
(recalled: MPE is not in this container).
"""
import os
import struct
import zlib

import numpy as np

AGENT = (0.35, 0.35, 0.85)
ADVERSARY = (0.85, 0.35, 0.35)
GOOD_TAG = (0.35, 0.85, 0.35)
LANDMARK = (0.25, 0.25, 0.25)
GOAL = (0.15, 0.65, 0.15)


def entity_table(sp):
    """[(size, rgb)] for agents then landmarks of scenario spec ``sp``."""
    n, na = sp.n_agents, sp.num_adversaries
    if sp.name == "simple":
        return [(0.05, LANDMARK), (0.05, (0.75, 0.75, 0.75))]
    if sp.name == "simple_spread":
        return [(0.15, AGENT)] * n + [(0.05, LANDMARK)] * n
    if sp.name == "simple_adversary":
        ents = [(0.15, ADVERSARY if i < na else AGENT) for i in range(n)]
        return ents + [(0.08, (0.15, 0.15, 0.15))] * (n - 1)
    if sp.name == "simple_tag":
        ents = [(0.075, ADVERSARY) if i < na else (0.05, GOOD_TAG) for i in range(n)]
        return ents + [(0.2, LANDMARK)] * 2
    raise ValueError(sp.name)


def rasterize(pos, table, goal=None, px=256, cam_range=1.0):
    """uint8 [px, px, 3] frame: white background, filled circles (later entities on top)."""
    img = np.ones((px, px, 3), np.float32)
    ys, xs = np.mgrid[0:px, 0:px]
    wx = (xs + 0.5) / px * 2 * cam_range - cam_range
    wy = cam_range - (ys + 0.5) / px * 2 * cam_range
    for k in range(len(table) - 1, -1, -1):            # agents drawn last (on top)
        size, rgb = table[k]
        if goal is not None and k == goal:
            rgb = GOAL
        m = (wx - pos[k, 0]) ** 2 + (wy - pos[k, 1]) ** 2 <= size * size
        img[m] = rgb
    return (img * 255 + 0.5).astype(np.uint8)


def write_png(path, rgb):
    h, w, _ = rgb.shape
    raw = b"".join(b"\x00" + rgb[r].tobytes() for r in range(h))

    def chunk(tag, data):
        c = struct.pack(">I", len(data)) + tag + data
        return c + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)
    png = (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)) +
           chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))
    with open(path, "wb") as f:
        f.write(png)


class FrameWriter:
    def __init__(self, out_dir, sp):
        self.dir = out_dir
        os.makedirs(out_dir, exist_ok=True)
        self.table = entity_table(sp)
        self.adversary_goal = sp.name == "simple_adversary"
        self.n_agents = sp.n_agents
        self.frames = []

    def add(self, pos, goal=0):
        """pos [n_entities, 2] of one env copy; goal = its goal landmark index"""
        g = self.n_agents + int(goal) if self.adversary_goal else None
        write_png(os.path.join(self.dir, f"frame_{len(self.frames):05d}.png"), rasterize(pos, self.table, g))
        self.frames.append(np.asarray(pos, np.float32).copy())

    def close(self):
        np.savez(os.path.join(self.dir, "positions.npz"), pos=np.stack(self.frames) if self.frames else np.zeros(0))
        return len(self.frames)
