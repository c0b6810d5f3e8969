"""Reference package path ``gentun.models`` (gentun/models/__init__.py)."""
