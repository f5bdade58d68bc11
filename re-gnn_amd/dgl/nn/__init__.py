from ..utils import expand_as_pair  # noqa: F401
from . import pytorch, functional  # noqa: F401
