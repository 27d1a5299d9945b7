"""Validation plots (reference `notebooks/New-Distributed-KMeans.ipynb:502-555`,
`notebooks/visualization.ipynb:189-199,336-346`): the first <= 10k points coloured by
label with the initial and final centers overlaid.  Written as self-contained SVG (no
plotting dependency); the first two feature columns are plotted."""
from __future__ import annotations

import numpy as np

PALETTE = ["#1f77b4", "#ff7f0e", "#2ca02c", "#d62728", "#9467bd", "#8c564b", "#e377c2",
           "#7f7f7f", "#bcbd22", "#17becf"]


def scatter_svg(path: str, x, labels=None, init_centers=None, centers=None,
                max_points: int = 10000, size: int = 640, title: str = "") -> str:
    x = np.asarray(x, dtype=np.float64)[:max_points, :2]
    lab = None if labels is None else np.asarray(labels)[:max_points]
    pts = [x]
    for c in (init_centers, centers):
        if c is not None:
            pts.append(np.asarray(c, dtype=np.float64)[:, :2])
    allp = np.concatenate(pts)
    finite = allp[np.isfinite(allp).all(1)]
    lo, hi = finite.min(0), finite.max(0)
    span = np.where(hi > lo, hi - lo, 1.0)
    pad = 20

    def tx(p):
        q = (p - lo) / span
        return pad + q[:, 0] * (size - 2 * pad), size - pad - q[:, 1] * (size - 2 * pad)

    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{size}" height="{size}">',
           f'<rect width="{size}" height="{size}" fill="white"/>']
    if title:
        out.append(f'<text x="{pad}" y="14" font-size="12">{title}</text>')
    px, py = tx(x)
    for i in range(len(x)):
        col = PALETTE[int(lab[i]) % len(PALETTE)] if lab is not None else "#444"
        out.append(f'<circle cx="{px[i]:.1f}" cy="{py[i]:.1f}" r="1.5" fill="{col}" fill-opacity="0.6"/>')
    for c, style in ((init_centers, 'fill="none" stroke="black"'), (centers, 'fill="black"')):
        if c is None:
            continue
        c = np.asarray(c, dtype=np.float64)[:, :2]
        ok = np.isfinite(c).all(1)
        cx, cy = tx(c[ok])
        for a, b in zip(cx, cy):
            out.append(f'<rect x="{a - 4:.1f}" y="{b - 4:.1f}" width="8" height="8" {style}/>')
    out.append("</svg>")
    with open(path, "w") as f:
        f.write("\n".join(out))
    return path
