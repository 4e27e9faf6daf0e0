"""Test-infrastructure oracle (see ``hdpissa_oracle.py`` header).  Not product code."""
from .hdpissa_oracle import *  # noqa: F401,F403
