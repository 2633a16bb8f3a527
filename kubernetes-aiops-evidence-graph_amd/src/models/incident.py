"""Mirror: `src.models.incident` is `egraph_dropin.models.incident` (the same module object)."""
import sys

import egraph_dropin.models.incident as _impl

sys.modules[__name__] = _impl
