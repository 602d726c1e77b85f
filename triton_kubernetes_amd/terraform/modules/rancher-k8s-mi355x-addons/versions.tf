terraform {
  required_version = ">= 1.4"
  required_providers {
    external = {
      source  = "hashicorp/external"
      version = ">= 2.0"
    }
    tls = {
      source  = "hashicorp/tls"
      version = ">= 4.0"
    }
  }
}
