"""seldon_core.microservice (``seldon-core-microservice``) -> seldon_core_amd.microservice."""
from seldon_core_amd.microservice import main  # noqa: F401

if __name__ == "__main__":
    main()
