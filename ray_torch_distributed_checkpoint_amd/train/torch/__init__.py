"""`ray.train.torch` equivalents: TorchTrainer, get_device, prepare_model, prepare_data_loader."""
from ..torch_utils import (enable_reproducibility, get_device, prepare_data_loader,  # noqa: F401
                           prepare_model)
from ..trainer import TorchTrainer  # noqa: F401
from ..config import TorchConfig  # noqa: F401
