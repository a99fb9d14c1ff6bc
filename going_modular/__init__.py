"""``going_modular`` compatibility package (reference going_modular/going_modular/*)."""
