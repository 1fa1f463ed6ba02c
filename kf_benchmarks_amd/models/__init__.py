"""Model zoo (registry in model_config)."""
