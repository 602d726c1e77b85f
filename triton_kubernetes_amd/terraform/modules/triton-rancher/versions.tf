terraform {
  required_version = ">= 1.4"
  required_providers {
    triton = {
      source  = "joyent/triton"
      version = ">= 0.8"
    }
    external = {
      source  = "hashicorp/external"
      version = ">= 2.0"
    }
  }
}
