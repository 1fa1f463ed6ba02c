"""Platform hooks (role of tcb/platforms/util.py): re-exports the default
platform; a site-specific platform replaces this import."""

from .default.util import *  # noqa: F401,F403
