from .flat import FlatParamSpace, space_of  # noqa: F401
from .fused import FusedAdamW, FusedSGD  # noqa: F401
from .overlap import BackwardOverlap  # noqa: F401
