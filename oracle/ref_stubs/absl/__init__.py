from . import flags  # noqa: F401
