"""Applications built on the clustering engine (reference notebooks' use cases)."""
