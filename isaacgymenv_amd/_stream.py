"""The current HIP stream of a device as the raw handle the C ABIs take (hipStream_t), without
torch.cuda.current_stream()'s Python device parsing and Stream object (~1.5 us per call on the
per-step host path: several calls per VecTask.step and PPO rollout step)."""
from __future__ import annotations

_index_cache = {}
_torch = None


def _t():
    global _torch
    if _torch is None:  # (imported on first use: the host-only importers of gymapi stay light)
        import torch
        _torch = torch
    return _torch


def _index(device) -> int:
    torch = _t()
    if device is None:
        return torch.cuda.current_device()
    idx = _index_cache.get(device)
    if idx is None:
        d = torch.device(device) if not isinstance(device, torch.device) else device
        idx = d.index if d.index is not None else torch.cuda.current_device()
        if isinstance(device, (str, torch.device)) and (not isinstance(device, torch.device) or d.index is not None):
            _index_cache[device] = idx  # (an index-less "cuda" follows the current device: not cached)
    return idx


def raw_stream(device=None) -> int:
    """torch.cuda.current_stream(device).cuda_stream, fast."""
    return _t()._C._cuda_getCurrentRawStream(_index(device))
