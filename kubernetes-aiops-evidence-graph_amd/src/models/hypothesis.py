"""Mirror: `src.models.hypothesis` is `egraph_dropin.models.hypothesis` (the same module object)."""
import sys

import egraph_dropin.models.hypothesis as _impl

sys.modules[__name__] = _impl
