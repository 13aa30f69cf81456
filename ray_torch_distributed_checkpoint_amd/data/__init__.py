from .dataset import Dataset, from_items, from_numpy  # noqa: F401
from .datasets import LABELS, SyntheticFashionMNIST, fashion_mnist, get_dataloaders, get_labels_map  # noqa: F401
