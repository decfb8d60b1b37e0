"""Model repository (layout, config.pbtxt schema, export / verify / sync)."""
from .model_config import ConfigError, generate, generate_pipeline, parse, validate  # noqa: F401
from .store import (  # noqa: F401
    PIPELINE,
    build_repository,
    init_flat,
    load_module,
    scan_repository,
    sync_repository,
    verify_repository,
)
