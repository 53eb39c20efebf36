"""Build, native loading, IO, timing and CLI helpers."""
