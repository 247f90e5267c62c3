"""Reference ``rocket/core/module.py``: Module."""

from rocket_amd.core.module import Module  # noqa: F401
