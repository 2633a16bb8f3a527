"""Mirror: `src.services.rca.rules_engine` is `egraph_dropin.rules_engine` (the same module object)."""
import sys

import egraph_dropin.rules_engine as _impl

sys.modules[__name__] = _impl
