"""Model front-ends (k-NN classifier, KD-tree)."""
