"""fqlpop -- MI355X-native Flow Q-Learning population trainer (HIP kernels behind a C ABI).

``Population`` is the engine; ``fql.agents.fql.FQLAgent`` and ``trainer.Trainer``
(sibling packages) keep the reference's surface on top of it.
"""
from fqlpop._lib import (EXPORTED_SYMBOLS, LIB_PATH, TRAIN_INFO_KEYS, VAL_INFO_KEYS,  # noqa: F401
                         FqlpopError, get_engine_option, is_diagnostic_build, load_library,
                         reset_engine_options, set_engine_option, step_streams)
from fqlpop.population import Population, PopulationConfig, split_plan  # noqa: F401
