"""Reference ``rocket/utils/collections.py``: collection traversal helpers."""

from rocket_amd.utils.collections import (  # noqa: F401
    apply_to_collection,
    apply_to_mapping,
    apply_to_sequence,
    is_collection,
)
