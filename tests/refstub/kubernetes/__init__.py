"""Test stand-in for the ``kubernetes`` package (see ../README.md)."""
from . import client, config  # noqa: F401
