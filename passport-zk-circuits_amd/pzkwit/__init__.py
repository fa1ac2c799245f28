"""pzkwit — MI355X-native batched witness generator for RegisterIdentityBuilder."""
