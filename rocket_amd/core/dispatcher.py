"""Ordered fan-out of lifecycle events to child capsules.

Parity (reference ``rocket/core/dispatcher.py``):

* children are validated (``ValueError`` on non-capsules, ``:198-223``) and sorted
  by ``_priority`` descending with a stable sort (``:54-56``);
* ``setup/set/reset/launch`` run the dispatcher's own ``Capsule`` handler first,
  then every child in order (``:58-76, :99-159``);
* ``destroy`` runs the children in **reverse** order, then itself (``:78-97``),
  which keeps the LIFO checkpoint-registration invariant;
* ``accelerate``/``clear`` propagate recursively (``:161-196``).
"""

from __future__ import annotations

from rocket_amd.core.attributes import Attributes
from rocket_amd.core.capsule import Capsule, Events


_BASE_DISPATCH = Capsule.dispatch  # a child whose dispatch differs (override, spy) keeps going through it


class Dispatcher(Capsule):
    def __init__(self, capsules: list[Capsule], priority: int = 1000) -> None:
        super().__init__(statefull=False, priority=priority)
        capsules = list(capsules)
        self.guard(capsules)
        # list.sort is stable: equal priorities keep insertion order
        self._capsules = sorted(capsules, key=lambda c: c._priority, reverse=True)
        self._launch_handlers = None  # (children list, bound launch handlers, len) — see launch(); set to None after re-binding a child's launch on the instance

    def _fan_out(self, event: Events, attrs: Attributes | None) -> None:
        for capsule in self._capsules:
            capsule.dispatch(event, attrs)

    def setup(self, attrs: Attributes | None = None) -> None:
        Capsule.setup(self, attrs=attrs)
        self._fan_out(Events.SETUP, attrs)

    def destroy(self, attrs: Attributes | None = None) -> None:
        for capsule in self._capsules[::-1]:
            capsule.dispatch(Events.DESTROY, attrs)
        Capsule.destroy(self, attrs=attrs)

    def set(self, attrs: Attributes | None = None) -> None:
        Capsule.set(self, attrs=attrs)
        self._fan_out(Events.SET, attrs)

    def reset(self, attrs: Attributes | None = None) -> None:
        Capsule.reset(self, attrs=attrs)
        self._fan_out(Events.RESET, attrs)

    def launch(self, attrs: Attributes | None = None) -> None:
        # the per-iteration event: the children's bound ``launch`` handlers, resolved once (a child
        # that overrides ``dispatch`` keeps going through it), called in priority order — the same
        # calls as ``_fan_out(Events.LAUNCH)`` without an enum lookup + getattr per child per step
        # (re-resolved when the child list is replaced or mutated in place: identity + length)
        hs = self._launch_handlers
        caps = self._capsules
        if hs is None or hs[0] is not caps or hs[2] != len(caps):
            hs = self._launch_handlers = (caps, [
                c.launch if type(c).dispatch is _BASE_DISPATCH else (lambda a, c=c: c.dispatch(Events.LAUNCH, a))
                for c in caps], len(caps))
        for h in hs[1]:
            h(attrs)

    def accelerate(self, accelerator) -> None:
        Capsule.accelerate(self, accelerator)
        for capsule in self._capsules:
            capsule.accelerate(accelerator)

    def clear(self) -> None:
        Capsule.clear(self)
        for capsule in self._capsules:
            capsule.clear()

    def guard(self, capsules: list[Capsule]) -> None:
        for capsule in capsules:
            if not isinstance(capsule, Capsule):
                raise ValueError(f"{self.__class__.__name__} got invalid capsule.")

    def iter_capsules(self, recursive: bool = True):
        """Yield children (depth-first when ``recursive``)."""
        for capsule in self._capsules:
            yield capsule
            if recursive and isinstance(capsule, Dispatcher):
                yield from capsule.iter_capsules(True)

    def __repr__(self) -> str:
        pad = " " * 4
        own = f"\n{pad}".join(
            f"{k}={str(v).replace(chr(10), chr(10) + pad * 2)}"
            for k, v in self.__dict__.items()
            if k != "_capsules"
        )
        kids = "\n".join(str(c) for c in self._capsules).replace("\n", f"\n{pad}")
        block = f"\n_capsules=[\n{pad}{kids}\n]".replace("\n", f"\n{pad}")
        return f"{self.__class__.__name__}(\n{pad}{own}{block}\n)"
