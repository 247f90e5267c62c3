"""Checkpoint writer/reader for the rocket on-disk layout.

The reference's ``Checkpointer`` calls ``accelerator.save_state(dir)``
(``rocket/core/checkpoint.py:129``) and ``Launcher._resume`` calls
``accelerator.load_state(dir)`` (``rocket/core/launcher.py:356-363``).  The
directory layout those produce is the compatibility contract:

    model.safetensors / model_{i}.safetensors   unwrapped state_dict, plain keys
    optimizer.bin / optimizer_{i}.bin           torch.save(optimizer.state_dict())
    scheduler.bin / scheduler_{i}.bin           torch.save(scheduler.state_dict())
    scaler.pt                                   fp16 GradScaler only
    random_states_{rank}.pkl                    python/numpy/torch(/cuda) RNG + GA step
    custom_checkpoint_{i}.pkl                   torch.save(obj.state_dict()), registration order

Loading rules kept: the number of ``custom_checkpoint_*.pkl`` files must equal
the number of registered objects (else ``RuntimeError``); a missing RNG file is
logged and skipped.  Files we read back are loaded with ``weights_only=True``
where their content allows it (model/optimizer/scheduler/custom state); the RNG
file stores numpy's RNG key as a tensor; reading an accelerate-written RNG file
allow-lists only numpy's array reconstruction.  Nothing is ever unpickled with
``weights_only=False``.
"""

from __future__ import annotations

import os
import random
import re
from pathlib import Path
from typing import List

import numpy as np
import torch
from safetensors.torch import load_file as st_load
from safetensors.torch import save_file as st_save

from rocket_amd.utils.logging import get_logger

logger = get_logger(__name__)

_CUSTOM_RE = re.compile(r"^custom_checkpoint_(\d+)\.pkl$")


def _suffixed(stem: str, ext: str, i: int) -> str:
    return f"{stem}{'' if i == 0 else f'_{i}'}.{ext}"


def _cpu_state_dict(model: torch.nn.Module) -> dict:
    out = {}
    seen = {}
    for k, v in model.state_dict().items():
        if not isinstance(v, torch.Tensor):
            continue
        t = v.detach()
        key = (t.untyped_storage().data_ptr(), t.storage_offset(), tuple(t.shape)) if t.numel() else None
        if key is not None and key in seen:  # tied weights: safetensors refuses shared storage
            continue
        if key is not None:
            seen[key] = k
        out[k] = t.to("cpu").contiguous().clone()
    return out


def _tied_aliases(model: torch.nn.Module) -> dict:
    """``{dropped key: kept key}`` for the tied entries :func:`_cpu_state_dict` leaves out."""
    seen, alias = {}, {}
    for k, v in model.state_dict().items():
        if not isinstance(v, torch.Tensor) or not v.numel():
            continue
        key = (v.untyped_storage().data_ptr(), v.storage_offset(), tuple(v.shape))
        if key in seen:
            alias[k] = seen[key]
        else:
            seen[key] = k
    return alias


def load_model_strict(model: torch.nn.Module, sd: dict, where: str = "checkpoint") -> None:
    """Load ``sd`` strictly (accelerate's ``load_state`` → safetensors ``load_model`` is strict too).

    The only keys allowed to be missing are tied aliases whose storage IS another loaded key
    (dropped at save time because safetensors refuses shared storage); every other missing or
    unexpected key raises, naming them — a checkpoint of another architecture never loads silently.
    """
    alias = _tied_aliases(model)
    missing, unexpected = model.load_state_dict(sd, strict=False)
    missing = [k for k in missing if not (k in alias and alias[k] in sd)]
    if missing or unexpected:
        raise RuntimeError(
            f"{where}: state dict does not match {type(model).__name__}: "
            f"missing keys {sorted(missing)[:20]}{' ...' if len(missing) > 20 else ''}, "
            f"unexpected keys {sorted(unexpected)[:20]}{' ...' if len(unexpected) > 20 else ''}"
        )


def _np_state_plain(st):
    # ('MT19937', uint32[624], pos, has_gauss, cached) with the key array as a tensor: weights_only-loadable
    return (st[0], torch.from_numpy(np.asarray(st[1], dtype=np.uint32).astype(np.int64)), int(st[2]), int(st[3]),
            float(st[4]))


def _np_state_restore(st):
    key = st[1]
    if isinstance(key, torch.Tensor):
        key = key.numpy().astype(np.uint32)
    return (st[0], np.asarray(key, dtype=np.uint32), int(st[2]), int(st[3]), float(st[4]))


def save_state(engine, output_dir: str) -> Path:
    out = Path(output_dir)
    out.mkdir(parents=True, exist_ok=True)
    # settle speculated scheduler steps before anything is written: a rolled-back step must leave
    # optimizer.bin (param-group lr) and scheduler.bin consistent
    for sched in engine._schedulers:
        sched._resolve()
    for i, model in enumerate(engine._models):
        st_save(_cpu_state_dict(engine.unwrap_model(model)), str(out / _suffixed("model", "safetensors", i)),
                metadata={"format": "pt"})
    for i, opt in enumerate(engine._optimizers):
        torch.save(opt.state_dict(), out / _suffixed("optimizer", "bin", i))
    for i, sched in enumerate(engine._schedulers):
        torch.save(sched.state_dict(), out / _suffixed("scheduler", "bin", i))
    if engine.scaler is not None:
        torch.save(engine.scaler.state_dict(), out / "scaler.pt")
    states = {
        "step": engine.step,
        "random_state": random.getstate(),
        "numpy_random_seed": _np_state_plain(np.random.get_state()),
        "torch_manual_seed": torch.get_rng_state(),
    }
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        states["torch_cuda_manual_seed"] = torch.cuda.get_rng_state_all()
    for i, obj in enumerate(engine._custom_objects):
        torch.save(obj.state_dict(), out / f"custom_checkpoint_{i}.pkl")
    # written last: its presence marks a complete checkpoint (Launcher.resume("latest"))
    torch.save(states, out / f"random_states_{engine.process_index}.pkl")
    return out


def _load(path, **kw):
    """Load with the restricted unpickler only — a checkpoint never executes code on resume."""
    try:
        return torch.load(path, weights_only=True, **kw)
    except Exception as e:
        raise RuntimeError(
            f"{path}: not loadable with torch.load(weights_only=True) ({e}). Checkpoint state must consist of "
            "tensors and plain Python containers/scalars."
        ) from e


def _numpy_safe_globals():
    """The numpy reconstruction entry points needed to read an RNG state array (no arbitrary code)."""
    out = [np.ndarray, np.dtype]
    for mod, name in (("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct")):
        try:
            m = __import__(mod, fromlist=[name])
            out.append(getattr(m, name))
        except Exception:
            pass
    try:
        out.append(type(np.dtype(np.uint32)))
    except Exception:
        pass
    return out


def custom_checkpoint_files(input_dir: str) -> List[str]:
    names = [f for f in os.listdir(input_dir) if _CUSTOM_RE.match(f)]
    return sorted(names, key=lambda f: int(_CUSTOM_RE.match(f).group(1)))


def load_state(engine, input_dir: str, load_custom: bool = True) -> None:
    src = Path(input_dir)
    if not src.is_dir():
        raise FileNotFoundError(f"checkpoint directory {input_dir} does not exist")
    for i, model in enumerate(engine._models):
        st = src / _suffixed("model", "safetensors", i)
        if st.exists():
            sd = st_load(str(st), device="cpu")
        else:
            sd = _load(src / _suffixed("pytorch_model", "bin", i), map_location="cpu")
        load_model_strict(engine.unwrap_model(model), sd, str(st if st.exists() else src))
    for i, opt in enumerate(engine._optimizers):
        opt.load_state_dict(_load(src / _suffixed("optimizer", "bin", i), map_location="cpu"))
    for i, sched in enumerate(engine._schedulers):
        sched.load_state_dict(_load(src / _suffixed("scheduler", "bin", i)))
    if engine.scaler is not None and (src / "scaler.pt").exists():
        engine.scaler.load_state_dict(_load(src / "scaler.pt"))
    rng = src / f"random_states_{engine.process_index}.pkl"
    if rng.exists():
        try:
            with torch.serialization.safe_globals(_numpy_safe_globals()):
                states = torch.load(rng, weights_only=True)
            engine.step = states.get("step", engine.step)
            random.setstate(states["random_state"])
            np.random.set_state(_np_state_restore(states["numpy_random_seed"]))
            torch.set_rng_state(states["torch_manual_seed"])
            if "torch_cuda_manual_seed" in states and torch.cuda.is_available():
                cuda_states = states["torch_cuda_manual_seed"]
                if len(cuda_states) == torch.cuda.device_count():
                    torch.cuda.set_rng_state_all(cuda_states)
        except Exception as e:  # pragma: no cover - mirrors accelerate's "could not load"
            logger.info(f"Could not load random states: {e}")
    else:
        logger.info("Could not load random states")
    if not load_custom:
        return
    files = custom_checkpoint_files(str(src))
    if len(files) != len(engine._custom_objects):
        raise RuntimeError(
            f"Number of custom checkpoints in folder {input_dir} does not match the number of registered objects:"
            f"\n\tFound checkpoints: {len(files)}\n\tRegistered objects: {len(engine._custom_objects)}\n"
        )
    for i, obj in enumerate(engine._custom_objects):
        obj.load_state_dict(_load(src / f"custom_checkpoint_{i}.pkl", map_location="cpu"))
