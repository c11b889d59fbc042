"""seldon_core.persistence -> seldon_core_amd.utils.persistence."""
from seldon_core_amd.utils.persistence import Persister as PersistenceThread  # noqa: F401
from seldon_core_amd.utils.persistence import persist, restore  # noqa: F401
