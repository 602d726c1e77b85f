"""cli package."""
