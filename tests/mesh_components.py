"""Python components placed on worker ranks by tests/fabric_worker.py."""
import numpy as np


class Doubler:
    """A TRANSFORMER that doubles every feature."""

    def transform_input(self, X, feature_names):
        return 2.0 * np.asarray(X, dtype=np.float64)


class Picky:
    """A TRANSFORMER that rejects rows with a negative first feature."""

    def transform_input(self, X, feature_names):
        X = np.asarray(X, dtype=np.float64)
        if (X[:, 0] < 0).any():
            raise ValueError("negative first feature")
        return X
