"""Command-line tools (clore-tx)."""
