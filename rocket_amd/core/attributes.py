"""The shared inter-capsule buffer.

Parity: reference ``rocket/core/capsule.py:23-35`` aliases ``adict`` — a dict whose
missing attributes read as ``None``.  ``adict`` is not installable here, so the
buffer is implemented natively.  Behaviour the capsules rely on:

* ``attrs.x`` for a missing key is ``None`` (never raises);
* ``attrs.x = v`` / ``del attrs.x`` map to item assignment / deletion;
* it is still a plain ``dict`` (``setdefault``, ``**`` unpacking, tqdm postfix);
* dunder lookups raise ``AttributeError`` so ``copy``/``pickle`` protocols keep working
  (a naive ``__getattr__ -> None`` breaks ``pickle`` and ``copy.deepcopy``).
"""

from __future__ import annotations

from typing import Any


class Attributes(dict):
    """``dict`` with attribute access; absent keys read as ``None``."""

    __slots__ = ()

    def __getattr__(self, name: str) -> Any:
        if name.startswith("__") and name.endswith("__"):
            raise AttributeError(name)
        return self.get(name)

    def __setattr__(self, name: str, value: Any) -> None:
        self[name] = value

    def __delattr__(self, name: str) -> None:
        try:
            del self[name]
        except KeyError:
            raise AttributeError(name) from None

    def __reduce__(self):
        return (type(self), (dict(self),))

    def __copy__(self) -> "Attributes":
        return type(self)(self)

    def __deepcopy__(self, memo) -> "Attributes":
        import copy

        out = type(self)()
        memo[id(self)] = out
        for k, v in self.items():
            out[copy.deepcopy(k, memo)] = copy.deepcopy(v, memo)
        return out

    def __repr__(self) -> str:
        return f"Attributes({dict.__repr__(self)})"
