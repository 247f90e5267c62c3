"""HIP runtime defaults for the step loop, applied before the runtime initialises.

Imported first by :mod:`rocket_amd`; every knob is a ``setdefault`` so an exported value wins.
Set ``ROCKET_HIP_DEFAULTS=0`` to leave the environment untouched.

``DEBUG_CLR_GRAPH_PACKET_CAPTURE=0`` — with packet capture on (the ROCm 7 default) a replayed
HIP graph submits its pre-built AQL packets as one batch, which is cheaper on the host but costs
the GPU ~4-5 µs of idle time at every graph boundary on MI355X.  A launch-bound step (the LeNet
headline: 5 kernels, ~60 µs of GPU work) is GPU-bound, so the per-node submission path wins:
measured on 1x MI355X, LeNet bs1024 0.0672 -> 0.0630 ms/step (15.2M -> 16.2M samples/s, two
alternating A/B runs each, ``scripts/gpu_envprobe2.sh``; ``profiles/r1_hip_env_ab.md``).  The
host pays ~5 µs more per replay, still below the GPU step time.

``ROCKET_DEBUG_SYNC=1`` (serialised debug mode) additionally sets
``AMD_SERIALIZE_KERNEL=3`` / ``AMD_SERIALIZE_COPY=3`` (the runtime waits for every kernel and copy
before the next) and ``HIP_LAUNCH_BLOCKING=1``; ``ops/_lib.check`` then synchronises after each
native launch, so a fault is attributed to the launch that caused it.
"""

import os

DEFAULTS = {
    "DEBUG_CLR_GRAPH_PACKET_CAPTURE": "0",
}


DEBUG = {
    "AMD_SERIALIZE_KERNEL": "3",
    "AMD_SERIALIZE_COPY": "3",
    "HIP_LAUNCH_BLOCKING": "1",
}


def apply() -> None:
    if os.environ.get("ROCKET_DEBUG_SYNC", "0") == "1":
        for k, v in DEBUG.items():
            os.environ.setdefault(k, v)
    if os.environ.get("ROCKET_HIP_DEFAULTS", "1") == "0":
        return
    for k, v in DEFAULTS.items():
        os.environ.setdefault(k, v)


apply()
