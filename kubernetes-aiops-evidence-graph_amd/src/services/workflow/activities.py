"""Mirror: `src.services.workflow.activities` is `egraph_dropin.activities` (the same module object)."""
import sys

import egraph_dropin.activities as _impl

sys.modules[__name__] = _impl
