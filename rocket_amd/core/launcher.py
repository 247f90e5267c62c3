"""Process / engine lifecycle and the epoch loop.

Parity (reference ``rocket/core/launcher.py``):

* constructor arguments (``:94-107``) and state ``{epoch_idx, num_procs,
  num_nodes}`` saved only when ``statefull`` (``:410-448``);
* project directory ``{logging_dir}/{tag}[/v{N}]`` with experiment versioning,
  rank 0 decides and broadcasts, existing dir without versioning raises
  (``:125-161``);
* ``launch`` = setup → resume → ``for epoch: capsule.set/launch/reset`` on the
  top-level capsules (called directly, not via dispatch) → destroy (``:255-287``);
* ``resume(path, load_capsules)`` records intent; the load happens inside
  ``launch`` after setup, and the distributed setup must match (``:319-408``);
* the ``notebook`` wrapper fills ``attrs.launcher`` and, inside a Jupyter
  kernel, spawns ``num_procs`` workers (``:202-247``).

Fixes: the process group is created before the
project-directory broadcast (Q9); ``load_capsules=False`` simply skips custom
objects instead of swapping the registry (Q10); the notebook path spawns with
``spawn`` (HIP cannot survive ``fork`` after init) using our own launcher.
"""

from __future__ import annotations

import os
import socket
from typing import Callable

from rocket_amd.core.attributes import Attributes
from rocket_amd.core.capsule import Capsule
from rocket_amd.core.dispatcher import Dispatcher
from rocket_amd.runtime import comm as _comm


def in_notebook() -> bool:
    try:
        from IPython import get_ipython  # noqa: F401

        ip = get_ipython()
        return ip is not None and "IPKernelApp" in ip.config
    except (ImportError, AttributeError):
        return False


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn_entry(local_rank: int, world: int, port: int, fn, args):
    os.environ.update(
        MASTER_ADDR="127.0.0.1",
        MASTER_PORT=str(port),
        RANK=str(local_rank),
        LOCAL_RANK=str(local_rank),
        WORLD_SIZE=str(world),
        LOCAL_WORLD_SIZE=str(world),
    )
    fn(*args)


def notebook_launch(fn: Callable, args=(), num_processes: int = 1) -> None:
    """Run ``fn(*args)`` on ``num_processes`` freshly spawned single-node workers."""
    if num_processes <= 1:
        fn(*args)
        return
    import torch.multiprocessing as mp

    mp.start_processes(_spawn_entry, args=(num_processes, _free_port(), fn, args), nprocs=num_processes,
                       start_method="spawn", join=True)


def notebook(method: Callable) -> Callable:
    """Decorator (reference ``Launcher.notebook``, ``launcher.py:202``): in a Jupyter kernel the
    wrapped ``method(self, attrs)`` runs on ``attrs.launcher.num_procs`` spawned workers, otherwise
    in-process.  ``Launcher.launch`` applies the same logic; this is for user launchers."""

    def wrapper(self, attrs: Attributes | None = None) -> None:
        attrs = attrs if attrs is not None else Attributes()
        if attrs.launcher is None:
            attrs.launcher = Attributes()
        attrs.launcher.setdefault("num_procs", getattr(self, "_num_procs", 1))
        attrs.launcher.setdefault("num_nodes", getattr(self, "_num_nodes", 1))
        if in_notebook() and (attrs.launcher.num_procs or 1) > 1:
            notebook_launch(method, args=(self, attrs), num_processes=attrs.launcher.num_procs)
        else:
            method(self, attrs)

    wrapper.__wrapped__ = method
    return wrapper


def latest_checkpoint(root: str) -> str | None:
    """Newest directory under ``root`` holding a complete checkpoint (``random_states_0.pkl`` is
    written last by the checkpoint writer), or None."""
    best, best_t = None, -1.0
    if not root or not os.path.isdir(root):
        return None
    for dirpath, _dirs, files in os.walk(root):
        if "random_states_0.pkl" in files:
            t = os.path.getmtime(os.path.join(dirpath, "random_states_0.pkl"))
            if t > best_t:
                best, best_t = dirpath, t
    return best


class Launcher(Dispatcher):
    def __init__(
        self,
        capsules: list[Capsule],
        tag: str | None = None,
        logging_dir: str = "./logs",
        experiment_versioning: bool = True,
        mixed_precision: str | None = None,
        gradient_accumulation_steps: int = 1,
        num_procs: int | None = 1,
        num_nodes: int | None = 1,
        num_epochs: int = 1,
        destroy_process_group_after_launch: bool = True,
        statefull: bool = False,
        seed: int | None = None,
        cpu: bool | None = None,
        engine_kwargs: dict | None = None,
    ) -> None:
        super().__init__(capsules=capsules)
        self._num_epochs = num_epochs
        self._epoch_idx = 0
        self._statefull = statefull
        self._num_procs = num_procs
        self._num_nodes = num_nodes
        self._mixed_precision = mixed_precision
        self._gradient_accumulation_steps = gradient_accumulation_steps
        self._tag = tag
        self._logging_dir = logging_dir
        self._experiment_versioning = experiment_versioning
        self._project_dir = None
        self._destroy_process_group_after_launch = destroy_process_group_after_launch
        self._resume_from = None
        self._load_capsules = True
        self._seed = seed
        self._cpu = cpu
        self._engine_kwargs = dict(engine_kwargs or {})

    # --------------------------------------------------------- project dir
    def _resolve_project_dir(self) -> None:
        if self._tag is None:
            return
        path = None
        if _comm.context().is_main_process:
            base = os.path.join(self._logging_dir, self._tag)
            if not self._experiment_versioning:
                if os.path.isdir(base):
                    path = ValueError(
                        "Project directory already exists and versioning is switched off. "
                        "Change experiment name or enable experiment versioning"
                    )
                else:
                    path = base
            else:
                versions = []
                if os.path.isdir(base):
                    for name in os.listdir(base):
                        if name.startswith("v") and name[1:].isdigit():
                            versions.append(int(name[1:]))
                path = os.path.join(base, f"v{max(versions, default=-1) + 1}")
        path = _comm.broadcast_object(path, src=0)
        if isinstance(path, Exception):
            raise path
        self._project_dir = path

    def _create_project_dir(self) -> None:
        if self._tag is None:
            return
        if _comm.context().is_main_process:
            os.makedirs(self._project_dir, exist_ok=True)
        _comm.barrier()

    # --------------------------------------------------------------- events
    def setup(self, attrs: Attributes | None = None) -> None:
        from rocket_amd.runtime.engine import Engine

        _comm.init(cpu=self._cpu)  # comm first (Q9)
        self._resolve_project_dir()
        engine = Engine(
            mixed_precision=self._mixed_precision,
            gradient_accumulation_steps=self._gradient_accumulation_steps,
            project_dir=self._project_dir,
            cpu=self._cpu,
            seed=self._seed,
            **self._engine_kwargs,
        )
        self.accelerate(engine)
        self._create_project_dir()
        self._num_procs = attrs.launcher.num_procs
        self._num_nodes = attrs.launcher.num_nodes
        attrs.launcher.world_size = engine.num_processes
        Dispatcher.setup(self, attrs)

    def set(self, attrs: Attributes | None = None) -> None:
        return None

    def reset(self, attrs: Attributes | None = None) -> None:
        return None

    notebook = staticmethod(notebook)

    def _notebook_entry(self, attrs: Attributes) -> None:
        self._run(attrs)

    def launch(self, attrs: Attributes | None = None) -> None:
        attrs = attrs if attrs is not None else Attributes()
        if attrs.launcher is None:
            attrs.launcher = Attributes()
        attrs.launcher.setdefault("num_procs", self._num_procs)
        attrs.launcher.setdefault("num_nodes", self._num_nodes)
        if in_notebook() and (attrs.launcher.num_procs or 1) > 1:
            notebook_launch(Launcher._notebook_entry, args=(self, attrs), num_processes=attrs.launcher.num_procs)
        else:
            self._run(attrs)

    def _run(self, attrs: Attributes) -> None:
        Capsule.launch(self, attrs)
        self.setup(attrs)
        self._resume(attrs)
        for epoch in range(self._epoch_idx, self._num_epochs):
            attrs.launcher.epoch_idx = epoch
            self._epoch_idx = epoch
            for capsule in self._capsules:
                capsule.set(attrs)
                capsule.launch(attrs)
                capsule.reset(attrs)
        self.destroy(attrs)

    @staticmethod
    def destroy_process_group() -> None:
        _comm.shutdown()

    def destroy(self, attrs: Attributes | None = None) -> None:
        Dispatcher.destroy(self, attrs=attrs)
        if attrs is not None and "launcher" in attrs:
            del attrs.launcher
        self._accelerator.end_training()
        self.clear()
        if self._destroy_process_group_after_launch:
            self.destroy_process_group()

    # --------------------------------------------------------------- resume
    def _resume(self, attrs: Attributes) -> None:
        if self._resume_from is None:
            return
        try:
            self._accelerator.load_state(self._resume_from, load_custom=self._load_capsules)
        except Exception as e:
            raise RuntimeError(
                "Failed to load state from resume checkpoint. Please check if the checkpoint is valid "
                f"and compatible with the current launcher configuration. ({e})"
            ) from e
        if self._num_procs != attrs.launcher.num_procs or self._num_nodes != attrs.launcher.num_nodes:
            raise RuntimeError("You need to resume your training in the exact same distributed setup.")

    def resume(self, path: str, load_capsules: bool = True) -> "Launcher":
        """Resume from a checkpoint directory; ``path="latest"`` picks the newest checkpoint written
        under ``logging_dir/tag`` by any previous version of this experiment (auto-resume)."""
        if path == "latest":
            path = latest_checkpoint(os.path.join(self._logging_dir, self._tag or ""))
            if path is None:
                self._logger.info("resume('latest'): no checkpoint found, starting fresh")
                return self
        self._resume_from = path
        self._load_capsules = load_capsules
        return self

    @property
    def project_dir(self) -> str | None:
        return self._project_dir

    def state_dict(self) -> dict:
        return dict(epoch_idx=self._epoch_idx, num_procs=self._num_procs, num_nodes=self._num_nodes)

    def load_state_dict(self, state: dict) -> None:
        self._epoch_idx = state["epoch_idx"]
        self._num_procs = state["num_procs"]
        self._num_nodes = state["num_nodes"]
