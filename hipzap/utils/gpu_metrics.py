"""Per-GPU utilisation for ``/metrics`` (SURVEY.md §5 metrics: "per-GPU utilization from amd-smi").

Read straight from the amdgpu driver's sysfs (``/sys/class/drm/card*/device``): busy percent,
VRAM used/total, power and edge temperature when exposed. A scrape costs a few file reads (no
subprocess; ``amd-smi metric`` takes ~100 ms), so /metrics can be polled every second. Cards
without the amdgpu files (or a container without /sys/class/drm) simply produce no samples.
"""
from __future__ import annotations

import glob
import os

_FILES = {
    "hipzap_gpu_busy_percent": "gpu_busy_percent",
    "hipzap_gpu_vram_used_bytes": "mem_info_vram_used",
    "hipzap_gpu_vram_total_bytes": "mem_info_vram_total",
}


def _read(path: str) -> float | None:
    try:
        with open(path) as f:
            return float(f.read().strip().split()[0])
    except (OSError, ValueError, IndexError):
        return None


def cards(root: str = "/sys/class/drm") -> list[str]:
    """amdgpu device directories, one per GPU (render nodes and connectors skipped)."""
    out = []
    for d in sorted(glob.glob(os.path.join(root, "card[0-9]*"))):
        dev = os.path.join(d, "device")
        if os.path.exists(os.path.join(dev, "gpu_busy_percent")):
            out.append(dev)
    return out


def sample(root: str = "/sys/class/drm") -> list[tuple[str, dict, float]]:
    """[(metric name, labels, value)] for every amdgpu card."""
    rows = []
    for i, dev in enumerate(cards(root)):
        lbl = {"gpu": str(i)}
        for name, fname in _FILES.items():
            v = _read(os.path.join(dev, fname))
            if v is not None:
                rows.append((name, lbl, v))
        for hw in glob.glob(os.path.join(dev, "hwmon", "hwmon*")):
            p = _read(os.path.join(hw, "power1_average")) or _read(os.path.join(hw, "power1_input"))
            if p is not None:
                rows.append(("hipzap_gpu_power_watts", lbl, p / 1e6))
            t = _read(os.path.join(hw, "temp1_input"))
            if t is not None:
                rows.append(("hipzap_gpu_temperature_celsius", lbl, t / 1e3))
            break
    return rows


def render(root: str = "/sys/class/drm") -> str:
    lines = []
    for name, lbl, v in sample(root):
        lab = ",".join(f'{k}="{x}"' for k, x in sorted(lbl.items()))
        lines.append(f"{name}{{{lab}}} {v:g}")
    return "\n".join(lines) + ("\n" if lines else "")
