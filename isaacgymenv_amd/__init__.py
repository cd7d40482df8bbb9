"""MI355X-native IsaacGymEnvs hot path.

HIP runtime setting applied before the runtime initialises: ``DEBUG_CLR_GRAPH_PACKET_CAPTURE=0``.
With graph packet capture on (the ROCm 7 default), a replayed HIP graph of the PPO minibatch
backward returned a wrong first-layer bias gradient on some replays (deterministically so under
AMD_SERIALIZE_KERNEL=3); with it off, every replay equals the eager gradient
(tools/probes/graph_bisect_probe.py, gpurun_out logs summarised in DESIGN.md).  ``GRAPHS_SAFE`` records
whether the setting is in force; the PPO learner only captures graphs when it is.
"""
import os as _os
import sys as _sys


def _graph_packet_capture_off() -> bool:
    if _os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE") == "0":
        return True
    torch = _sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():
        return False  # the runtime already read its environment
    _os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] = "0"
    return True


GRAPHS_SAFE = _graph_packet_capture_off()
