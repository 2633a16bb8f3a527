"""Mirror: `src.services.rca.hypothesis_ranker` is `egraph_dropin.hypothesis_ranker` (the same module object)."""
import sys

import egraph_dropin.hypothesis_ranker as _impl

sys.modules[__name__] = _impl
