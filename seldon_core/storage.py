"""seldon_core.storage -> seldon_core_amd.utils.storage."""
from seldon_core_amd.utils.storage import Storage  # noqa: F401
