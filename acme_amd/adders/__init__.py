"""Adders: pack environment interaction into replay items (acme/adders)."""
from acme_amd.adders.base import Adder  # noqa: F401
