"""seldon_core.serving_test_gen -> seldon_core_amd.testers."""
from seldon_core_amd.testers import create_seldon_api_testing_file  # noqa: F401
