"""readiness package."""
