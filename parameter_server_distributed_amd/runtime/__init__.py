"""runtime."""
