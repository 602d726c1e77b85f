"""node package."""
