"""Mirror of the hot path's models (reference src/models/__init__.py): egraph_dropin.models."""
from egraph_dropin.models import *  # noqa: F401,F403
from egraph_dropin.models import __all__  # noqa: F401
