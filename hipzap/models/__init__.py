from . import registry  # noqa: F401
from . import resnet  # noqa: F401
