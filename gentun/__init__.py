"""Import-name alias so code written against the reference (``from gentun
import ...``, README examples) runs unchanged on gentun_amd."""

from gentun_amd import *  # noqa: F401,F403
from gentun_amd import __all__, __version__  # noqa: F401
