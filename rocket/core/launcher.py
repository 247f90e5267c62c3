"""Reference ``rocket/core/launcher.py``: Launcher, in_notebook."""

from rocket_amd.core.launcher import Launcher, in_notebook, latest_checkpoint, notebook  # noqa: F401
