"""Reference ``rocket/utils/torch.py``: collate / device-move helpers."""

from rocket_amd.utils.torch import (  # noqa: F401
    BUILTIN_TYPES,
    move,
    register_default_move_hook,
    register_move_hook,
    torch_collate,
    torch_move,
)
