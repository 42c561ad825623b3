"""Model front-ends (exact k-NN classifier, serial KD-tree)."""
from .knn_classifier import KDTree, KNNClassifier  # noqa: F401
