terraform {
  required_version = ">= 1.3"
}
