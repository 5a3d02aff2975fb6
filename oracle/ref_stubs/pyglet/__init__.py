"""pyglet stub (rendering is out of scope)."""
from . import image  # noqa: F401
