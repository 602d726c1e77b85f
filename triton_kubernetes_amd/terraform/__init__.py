"""terraform package."""
