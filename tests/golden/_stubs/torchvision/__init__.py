"""Import-satisfying placeholder for torchvision (only the CNN-ESC50 path, out of scope, uses it)."""
from . import transforms  # noqa: F401
