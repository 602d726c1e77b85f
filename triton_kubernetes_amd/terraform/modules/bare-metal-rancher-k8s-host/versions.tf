terraform {
  required_version = ">= 1.4"
}
