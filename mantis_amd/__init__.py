"""mantis_amd — MI355X-native mantis3 hot path."""
