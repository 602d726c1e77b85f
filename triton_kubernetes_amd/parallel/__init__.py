"""parallel package."""
