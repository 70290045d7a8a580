"""Small shared helpers (size parsing, logging)."""
from .sizes import parse_size, format_mib  # noqa: F401
from .log import get_logger  # noqa: F401
