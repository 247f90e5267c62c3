"""Capsule protocol: lifecycle events and the base class every component derives from.

Parity map (reference ``rocket/core/capsule.py``):

* ``Events`` values are the handler method names (``:64-68``); ``dispatch`` calls
  ``getattr(self, event.value)(attrs)`` (``:254``).
* ``Capsule(statefull, logger, priority)`` (``:104-114``).
* ``setup`` checks the runtime engine and, for stateful capsules, registers the
  capsule for checkpointing (``:116-141``).  ``destroy`` enforces the strict LIFO
  unregistration invariant (``:143-176``).
* ``accelerate``/``clear``/``check_accelerator``/``set_logger``/``state_dict``/
  ``load_state_dict``/``__repr__`` (``:256-440``).

Differences (bug fixes): a capsule remembers whether it was
actually registered, so a stateful capsule that skipped ``Capsule.setup`` (the
reference ``Checkpointer``, Q1) destroys cleanly instead of popping somebody
else's registration.

The attribute that holds the runtime is still called ``_accelerator`` and is set
through ``accelerate(engine)`` so user capsules written against the reference
keep working; the object stored there is a :class:`rocket_amd.runtime.Engine`.
"""

from __future__ import annotations

import logging
from enum import Enum
from typing import Any

from rocket_amd.core.attributes import Attributes
from rocket_amd.utils.logging import get_logger


class Events(Enum):
    """Lifecycle events; the value is the name of the handler invoked."""

    SETUP = "setup"
    DESTROY = "destroy"
    SET = "set"
    RESET = "reset"
    LAUNCH = "launch"


class Capsule:
    """Base component of a rocket pipeline.

    Handlers (``setup``, ``destroy``, ``set``, ``reset``, ``launch``) all take the
    shared :class:`Attributes` buffer (or ``None``).
    """

    def __init__(
        self,
        statefull: bool = False,
        logger: logging.Logger | None = None,
        priority: int = 1000,
    ) -> None:
        super().__init__()
        self._priority = priority
        self._statefull = statefull
        self._accelerator = None
        self._registered = False
        self._logger = logger or get_logger(self.__module__)

    # ------------------------------------------------------------------ events
    def setup(self, attrs: Attributes | None = None) -> None:
        self.check_accelerator()
        if self._statefull:
            self._accelerator.register_for_checkpointing(self)
            self._registered = True
        self._logger.debug(f"{self.__class__.__name__} initialized.")

    def destroy(self, attrs: Attributes | None = None) -> None:
        if self._statefull and self._registered:
            objects = self._accelerator._custom_objects
            obj = objects.pop() if objects else None
            if obj is not self:
                if obj is not None:
                    objects.append(obj)
                raise RuntimeError(
                    f"{self.__class__.__name__}: Illegal destroy request. "
                    f"Attempted to remove {obj.__class__.__name__}, "
                    f"but expected {self.__class__.__name__}."
                )
            self._registered = False
        self._logger.debug(f"{self.__class__.__name__} destroyed.")

    def launch(self, attrs: Attributes | None = None) -> None:
        return None

    def set(self, attrs: Attributes | None = None) -> None:
        return None

    def reset(self, attrs: Attributes | None = None) -> None:
        return None

    def dispatch(self, event: Events, attrs: Attributes | None = None) -> Any:
        return getattr(self, event.value)(attrs)

    # ----------------------------------------------------------------- runtime
    def accelerate(self, accelerator) -> None:
        """Attach the runtime engine (name kept for reference API parity)."""
        self._accelerator = accelerator

    @property
    def engine(self):
        return self._accelerator

    def clear(self) -> None:
        self._accelerator = None

    def set_logger(self, logger: logging.Logger) -> None:
        self._logger = logger

    def check_accelerator(self) -> None:
        if self._accelerator is None:
            raise RuntimeError(
                f"{self.__class__.__name__}: accelerator is not defined. "
                "Please, specify it in __init__ function "
                "or set it via .accelerate(accelerator) method."
            )

    # ------------------------------------------------------------------ state
    def state_dict(self) -> dict:
        if not self._statefull:
            return {}
        raise NotImplementedError("state_dict() must be implemented by stateful subclasses")

    def load_state_dict(self, state_dict: dict) -> None:
        if not self._statefull:
            return
        raise NotImplementedError("load_state_dict() must be implemented by subclasses")

    def __repr__(self) -> str:
        pad = " " * 4
        fields = f"\n{pad}".join(
            f"{k}={str(v).replace(chr(10), chr(10) + pad * 2)}" for k, v in self.__dict__.items()
        )
        return f"{self.__class__.__name__}(\n{pad}{fields}\n)"
