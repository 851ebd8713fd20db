from .box import Box  # noqa: F401
from .multi_discrete import MultiDiscrete  # noqa: F401
from . import box, multi_discrete  # noqa: F401
