"""Mirror: `src.models.evidence` is `egraph_dropin.models.evidence` (the same module object)."""
import sys

import egraph_dropin.models.evidence as _impl

sys.modules[__name__] = _impl
