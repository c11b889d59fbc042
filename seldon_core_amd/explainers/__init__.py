"""Model explainers: anchor explanations for tabular, text and
image models, served next to a predictor by ``explainers.server``."""
from .anchor import AnchorImage, AnchorSearch, AnchorTabular, AnchorText, grid_slic

__all__ = ["AnchorImage", "AnchorSearch", "AnchorTabular", "AnchorText", "grid_slic"]
