"""Platform layer (the Azure Container Apps environment equivalent)."""
